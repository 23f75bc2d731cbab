"""Co-run observations from per-pod kernel traces: the deployed producer of the co-run
model's online learning.

The reference's recommender follows its data by retraining when the training files change
(reference pkg/recommender/recom_server.py:74-134); nothing in a running cluster feeds it.
Here the node agent already ingests every webhook-profiled pod's rocprofv3 kernel trace
(agent.pod_profiler.ProfileIngestor).  This observer turns those traces into what the co-run
model (models.corun.OnlineCorun, served by the recommender's ObserveCorun) learns from:

  * each traced pod contributes its kernel interval [first kernel start, last kernel end] on
    its device (the scheduler's device annotation; rocprofv3's timestamps share one node-wide
    clock, so intervals of different pods compare);
  * a pod becomes an observation (the group's target) once its co-runners are known: the
    pods on the same device UUID whose intervals overlap its own, pinned at their measured
    intervals (the target is predicted given what they really did), with start offsets;
  * co-runners still running when the target is ingested are waited for: the pods running on
    the device then (`running_on`) must all have finished, and a target whose co-runner
    finished without a trace (not profiled) is dropped -- its pressure would be missing from
    the group and bias the fit;
  * co-runners that had ALREADY finished when the target was ingested are found by their
    container times (`finished_on`: terminal pods on the device whose container
    startedAt .. finishedAt overlaps the target's own container span); any of them without a
    trace drops the target for the same reason.

A pod that ran ALONE on its device becomes a 1-pod group: for a workload the co-run model
does not know yet, the recommender cold-starts its row from it (models.coldstart).

Observations go to the recommender in batches (`send`, e.g. RecommenderClient.observe_corun);
its refit worker then serves a new ExportTable("corun") version, which the schedulers'
CachedPredictions pick up on their next refresh.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Any, Callable, Dict, List, Optional, Set, Tuple

from ..api import constants as C
from ..api import objects as O

log = logging.getLogger(__name__)


class CorunObserver:
    def __init__(self, send: Callable[[List[Dict[str, Any]]], Any],
                 running_on: Optional[Callable[[str], Set[str]]] = None, settle_s: float = 5.0,
                 clock: Callable[[], float] = time.monotonic, keep_s: float = 900.0, max_group: int = 16,
                 finished_on: Optional[Callable[[str, Tuple[float, float]], Set[str]]] = None):
        self.send = send
        self.running_on = running_on
        self.finished_on = finished_on
        self.settle_s = settle_s
        self.clock = clock
        self.keep_s = keep_s
        self.max_group = max_group
        self._lock = threading.Lock()
        self._recs: Dict[str, List[Dict[str, Any]]] = {}          # device uuid -> records
        self.sent = 0
        self.dropped = 0
        self.last_reply: Any = None

    @staticmethod
    def device_of(pod: Dict[str, Any]) -> Optional[str]:
        """The pod's single device (the scheduler's assignment annotation); None for a pod
        without one or on several devices (not one co-run group)."""
        devs = [d for d in (O.annotations(pod).get(C.ANNOT_DEVICES) or "").split(",") if d]
        return devs[0] if len(devs) == 1 else None

    def add(self, pod: Dict[str, Any], workload: str, iters: float, first_ns: int, last_ns: int,
            mfma_share: Optional[float] = None, cu_fill: Optional[float] = None) -> bool:
        uuid = self.device_of(pod)
        if uuid is None or last_ns <= first_ns:
            return False
        key = O.key(pod)
        running = None
        if self.running_on is not None:
            running = set(self.running_on(uuid)) - {key}
        if self.finished_on is not None:
            from ..plugins.gpu.feedback import container_span
            span = container_span(pod)
            if span is not None:
                # (never running any more: _ready then only asks that each left a trace)
                running = (running or set()) | (set(self.finished_on(uuid, span)) - {key})
        with self._lock:
            self._recs.setdefault(uuid, []).append(
                {"key": key, "workload": workload, "iters": float(iters), "s": int(first_ns), "e": int(last_ns),
                 "t": self.clock(), "wait": running, "emitted": False,
                 "mfma": -1.0 if mfma_share is None else float(mfma_share),
                 "fill": -1.0 if cu_fill is None else float(cu_fill)})
        return True

    def _ready(self, uuid: str, r: Dict[str, Any], traced: Set[str]) -> Optional[bool]:
        """True: emit; False: drop; None: not yet."""
        if self.clock() - r["t"] < self.settle_s:
            return None
        if r["wait"] is None:
            return True
        if self.running_on is not None and r["wait"] & set(self.running_on(uuid)):
            return None                     # a co-runner of it is still running
        return r["wait"] <= traced          # every one of them left a trace

    def step(self) -> int:
        """Emit every ready observation; returns how many were sent."""
        out: List[Dict[str, Any]] = []
        with self._lock:
            items = {u: list(rs) for u, rs in self._recs.items()}
        for uuid, rs in items.items():
            traced = {r["key"] for r in rs}
            for r in rs:
                if r["emitted"] or r["iters"] <= 0:
                    continue
                ok = self._ready(uuid, r, traced)
                if ok is None:
                    continue
                r["emitted"] = True
                if not ok:
                    self.dropped += 1
                    continue
                mem = [x for x in rs if x["e"] > r["s"] and x["s"] < r["e"]]
                if len(mem) > self.max_group:
                    self.dropped += 1
                    continue
                t0 = min(x["s"] for x in mem)
                out.append({"workloads": [x["workload"] for x in mem],
                            "iters": [x["iters"] if x["iters"] > 0 else 1.0 for x in mem],
                            "ms": [(x["e"] - x["s"]) / 1e6 for x in mem],
                            "start_ms": [(x["s"] - t0) / 1e6 for x in mem],
                            "target": [x is r for x in mem],
                            # per member: MFMA share of its kernel time (-1 unknown); a 1-pod
                            # group of an unseen workload cold-starts its co-run row
                            "mfma_share": [x.get("mfma", -1.0) for x in mem],
                            # ... and the CU fill of its kernels (-1 unknown)
                            "cu_fill": [x.get("fill", -1.0) for x in mem]})
        sent = 0
        if out:
            try:
                self.last_reply = self.send(out)
                sent = len(out)
                self.sent += sent
            except Exception as e:           # recommender down: these observations are lost
                log.warning("co-run observations not delivered: %s", e)
        self._prune()
        return sent

    def _prune(self) -> None:
        now = self.clock()
        with self._lock:
            for uuid, rs in list(self._recs.items()):
                keep = [r for r in rs if not r["emitted"] or now - r["t"] < self.keep_s]
                if keep:
                    self._recs[uuid] = keep
                else:
                    del self._recs[uuid]

    def pending(self) -> int:
        with self._lock:
            return sum(1 for rs in self._recs.values() for r in rs if not r["emitted"] and r["iters"] > 0)
