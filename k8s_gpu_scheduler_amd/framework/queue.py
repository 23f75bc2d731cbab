"""Scheduling queue: activeQ (priority heap), backoffQ, unschedulable pods.

Same structure as upstream kube-scheduler's PriorityQueue (inside the binary the
reference links, reference cmd/scheduler/main.go:20-22): pods failing a cycle go to the
unschedulable map and are moved back on cluster events (node add/update, pod delete) or
after a timeout, with exponential per-pod backoff.
"""
from __future__ import annotations

import functools
import heapq
import itertools
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..api import objects as O

Obj = Dict[str, Any]


@dataclass
class QueuedPodInfo:
    pod: Obj
    timestamp: float = field(default_factory=time.monotonic)
    attempts: int = 0
    initial_attempt: float = 0.0
    unschedulable_plugins: set = field(default_factory=set)
    cycle: int = 0                  # scheduling cycle in which it was last popped


class SchedulingQueue:
    def __init__(self, less: Optional[Callable[[QueuedPodInfo, QueuedPodInfo], bool]] = None,
                 initial_backoff_s: float = 1.0, max_backoff_s: float = 10.0,
                 unschedulable_timeout_s: float = 60.0,
                 sort_key: Optional[Callable[[QueuedPodInfo], Any]] = None):
        """`sort_key` (optional, the queueSort plugin's total-order form of `less`): the
        active heap then holds (key, seq, pod info) tuples compared in C, with the key
        evaluated once per push instead of in every comparison."""
        self._less = less or (lambda a, b: a.timestamp < b.timestamp)
        self._sort_key = sort_key
        self._cv = threading.Condition()
        self._seq = itertools.count()
        self._active: List[Any] = []
        self._active_keys: Dict[str, QueuedPodInfo] = {}
        self._backoff: List[Any] = []
        self._backoff_keys: Dict[str, QueuedPodInfo] = {}
        self._unsched: Dict[str, QueuedPodInfo] = {}
        self._in_flight: set = set()
        self.initial_backoff_s = initial_backoff_s
        self.max_backoff_s = max_backoff_s
        self.unschedulable_timeout_s = unschedulable_timeout_s
        self._closed = False
        # upstream's schedulingCycle / moveRequestCycle: a move request (cluster event) that
        # happens WHILE a pod is being scheduled must not be lost when that pod then fails --
        # e.g. preemption deletes victims inside the preemptor's own cycle
        self._cycle = 0
        self._move_request_cycle = -1
        less_fn = self._less

        @functools.total_ordering
        class _Item:
            __slots__ = ("pi", "seq")

            def __init__(self, pi, seq):
                self.pi, self.seq = pi, seq

            def __lt__(self, other):
                if less_fn(self.pi, other.pi):
                    return True
                if less_fn(other.pi, self.pi):
                    return False
                return self.seq < other.seq

            def __eq__(self, other):
                return self.seq == other.seq
        self._Item = _Item

    # ---------------------------------------------------------------- helpers
    def _backoff_duration(self, pi: QueuedPodInfo) -> float:
        d = self.initial_backoff_s * (2 ** max(pi.attempts - 1, 0))
        return min(d, self.max_backoff_s)

    def _push_active(self, pi: QueuedPodInfo) -> None:
        k = O.key(pi.pod)
        self._active_keys[k] = pi
        if self._sort_key is not None:
            heapq.heappush(self._active, (self._sort_key(pi), next(self._seq), pi))
        else:
            heapq.heappush(self._active, self._Item(pi, next(self._seq)))

    def _flush_backoff(self) -> None:
        now = time.monotonic()
        while self._backoff and self._backoff[0][0] <= now:
            _, _, pi = heapq.heappop(self._backoff)
            k = O.key(pi.pod)
            if self._backoff_keys.get(k) is pi:
                del self._backoff_keys[k]
                self._push_active(pi)
        for k, pi in list(self._unsched.items()):
            if now - pi.timestamp > self.unschedulable_timeout_s:
                del self._unsched[k]
                self._push_active(pi)

    # ---------------------------------------------------------------- API
    def add(self, pod: Obj) -> None:
        with self._cv:
            k = O.key(pod)
            self._unsched.pop(k, None)
            self._backoff_keys.pop(k, None)
            if k in self._active_keys:
                self._active_keys[k].pod = pod
            else:
                self._push_active(QueuedPodInfo(pod))
            self._cv.notify()

    def add_many(self, pods: List[Obj]) -> None:
        with self._cv:
            for pod in pods:
                k = O.key(pod)
                if k not in self._active_keys:
                    self._push_active(QueuedPodInfo(pod))
            self._cv.notify_all()

    def update(self, pod: Obj) -> None:
        with self._cv:
            k = O.key(pod)
            for d in (self._active_keys, self._backoff_keys, self._unsched):
                if k in d:
                    d[k].pod = pod
                    if d is self._unsched:       # an update may make it schedulable
                        pi = self._unsched.pop(k)
                        self._push_active(pi)
                        self._cv.notify()
                    return
            if k not in self._in_flight:
                self._push_active(QueuedPodInfo(pod))
                self._cv.notify()

    def delete(self, pod: Obj) -> None:
        with self._cv:
            k = O.key(pod)
            self._active_keys.pop(k, None)     # heap entries are lazily skipped
            self._backoff_keys.pop(k, None)
            self._unsched.pop(k, None)

    def pop(self, timeout_s: Optional[float] = None) -> Optional[QueuedPodInfo]:
        deadline = None if timeout_s is None else time.monotonic() + timeout_s
        with self._cv:
            while True:
                self._flush_backoff()
                while self._active:
                    item = heapq.heappop(self._active)
                    pi = item[2] if type(item) is tuple else item.pi
                    k = O.key(pi.pod)
                    if self._active_keys.get(k) is pi:
                        del self._active_keys[k]
                        pi.attempts += 1
                        self._cycle += 1
                        pi.cycle = self._cycle
                        if not pi.initial_attempt:
                            pi.initial_attempt = time.monotonic()
                        self._in_flight.add(k)
                        return pi
                if self._closed:
                    return None
                wait = 0.05
                if deadline is not None:
                    rem = deadline - time.monotonic()
                    if rem <= 0:
                        return None
                    wait = min(wait, rem)
                if self._backoff:
                    wait = min(wait, max(0.0, self._backoff[0][0] - time.monotonic()))
                self._cv.wait(wait)

    def done(self, pod: Obj) -> None:
        with self._cv:
            self._in_flight.discard(O.key(pod))

    def add_unschedulable(self, pi: QueuedPodInfo, backoff: bool = True) -> None:
        with self._cv:
            k = O.key(pi.pod)
            self._in_flight.discard(k)
            pi.timestamp = time.monotonic()
            if backoff and self._move_request_cycle >= pi.cycle > 0:
                exp = pi.timestamp + self._backoff_duration(pi)
                self._backoff_keys[k] = pi
                heapq.heappush(self._backoff, (exp, next(self._seq), pi))
                self._cv.notify()
            elif backoff:
                self._unsched[k] = pi
            else:
                self._push_active(pi)
                self._cv.notify()

    def move_all_to_active_or_backoff(self, event: str = "") -> None:
        with self._cv:
            self._move_request_cycle = self._cycle
            now = time.monotonic()
            for k, pi in list(self._unsched.items()):
                del self._unsched[k]
                exp = pi.timestamp + self._backoff_duration(pi)
                if exp > now:
                    self._backoff_keys[k] = pi
                    heapq.heappush(self._backoff, (exp, next(self._seq), pi))
                else:
                    self._push_active(pi)
            self._cv.notify_all()

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()

    def active_pods(self) -> List[Obj]:
        """Pods waiting in the active queue (not the one being scheduled), in no order."""
        with self._cv:
            return [pi.pod for pi in self._active_keys.values()]

    def pending(self) -> Dict[str, int]:
        with self._cv:
            return {"active": len(self._active_keys), "backoff": len(self._backoff_keys),
                    "unschedulable": len(self._unsched)}

    def __len__(self) -> int:
        with self._cv:
            return len(self._active_keys) + len(self._backoff_keys) + len(self._unsched)
