"""Measured backlog feedback for the burst planner in a deployed cluster.

The planner's backlog carry (plugins.gpu.planner, `planCarry`) remembers how much predicted
work each GPU took beyond the least-loaded one, so the SLO phase's slack does not random-walk
onto one GPU.  In the bench, each collected epoch corrects that backlog with the GPU's
measured busy time.  A cluster has no epochs -- but every batch pod ends, and its end is
observable: the kubelet reports each container's `startedAt` / `finishedAt`.

A raw measured / predicted ratio is useless as a correction: a container's wall time includes
process start, model loading and host work the co-run model's GPU time does not, so every
ratio is far above 1 and the backlog would drown.  What matters for placement is whether one
GPU runs SLOWER THAN ITS SIBLINGS relative to the model (a GPU with a degraded link, a lower
clock under a power cap, a noisy neighbour outside Kubernetes, or the model's error on the
mix it gets).  So each completion is normalised by the node-wide median ratio of recent
completions:

    delta_ms(pod) = measured_ms / median_ratio  -  predicted_ms

and the GPU's co-run group gets `planner.observe_time(group, predicted, measured / median)`:
the planner keeps a window median of those ratios per GPU as its measured speed and scales the
GPU's future backlog increments by it (bounded -- see BurstPlanner.observe_time).  A uniform
slowdown of every GPU moves the median, not the speeds; one slow GPU's pods come out above
the median and shift the next plans off it.

Predicted durations are recorded at Reserve (the pod's group on the co-run model, with the
residents it was placed next to); completions arrive through the pod informer (the GPU
plugin's `_on_pod`).  The measurement is `gpu-scheduler.amd.com/busy-ms` when the pod carries
it: the node agent writes it on every pod that terminates on its GPUs, from amd-smi's
per-process GPU engine time summed over the pod's processes, or from the rocprof trace of a
profiled pod (agent.busy.BusyTracker).  Otherwise the containers' startedAt .. finishedAt --
but the kubelet serialises those at WHOLE SECONDS (RFC 3339 without a fraction), so a span
shorter than QUANTISED_MIN_SPAN_S is quantisation noise (a 2-s pod reads anything from 1 to 3
s) and is not fed at all.

Reference analog: the reference's Score reads resident state every cycle but never learns
from completions (reference pkg/plugins/gpu_plugin/gpu_plugins.go:87-160, 558-757).
"""
from __future__ import annotations

import collections
import datetime as _dt
import statistics
import threading
from typing import Any, Dict, Hashable, List, Optional, Tuple

from ...api import constants as C
from ...api import objects as O

Obj = Dict[str, Any]
ANNOT_BUSY_MS = C.ANNOT_PREFIX + "busy-ms"
# whole-second container timestamps: spans shorter than this are not measurements (+-1 s of
# quantisation is > 5 % below 20 s)
QUANTISED_MIN_SPAN_S = 20.0


def _ts(s: str) -> Optional[float]:
    """RFC 3339 (the kubelet's `2024-01-01T00:00:00Z`, fractional seconds allowed) -> epoch s."""
    if not s:
        return None
    try:
        if s.endswith("Z"):
            s = s[:-1] + "+00:00"
        return _dt.datetime.fromisoformat(s).timestamp()
    except ValueError:
        return None


def measured_ms(pod: Obj) -> Optional[float]:
    """The pod's measured run time: the busy-ms annotation, else its containers' span
    (earliest startedAt .. latest finishedAt of terminated containers)."""
    ann = O.annotations(pod).get(ANNOT_BUSY_MS)
    if ann:
        try:
            v = float(ann)
            if v > 0:
                return v
        except ValueError:
            pass
    span = container_span(pod, QUANTISED_MIN_SPAN_S)
    return None if span is None else (span[1] - span[0]) * 1e3


def _whole_seconds(s: str) -> bool:
    """An RFC 3339 time without a fractional second (the kubelet's serialisation)."""
    return "." not in s.split("T")[-1]


def container_span(pod: Obj, min_quantised_s: float = 0.0) -> Optional[Tuple[float, float]]:
    """(earliest startedAt, latest finishedAt) of the pod's terminated containers, epoch s.
    None when a span built from whole-second timestamps is shorter than `min_quantised_s`."""
    t0, t1 = None, None
    coarse = True               # every timestamp whole-second (one with a fraction: fine-grained)
    for cs in (pod.get("status") or {}).get("containerStatuses") or []:
        term = (cs.get("state") or {}).get("terminated") or {}
        sa, sb = term.get("startedAt", ""), term.get("finishedAt", "")
        a, b = _ts(sa), _ts(sb)
        if a is None or b is None or b < a:
            continue
        coarse = coarse and _whole_seconds(sa) and _whole_seconds(sb)
        t0 = a if t0 is None else min(t0, a)
        t1 = b if t1 is None else max(t1, b)
    if t0 is None or t1 is None or t1 <= t0:
        return None
    if coarse and t1 - t0 < min_quantised_s:
        return None
    return t0, t1


class CompletionFeedback:
    """window: recent completions the node-wide median ratio is taken over; min_n: no
    correction before that many (the median of a handful is noise)."""

    def __init__(self, planner: Any, window: int = 64, min_n: int = 8, max_pending: int = 4096):
        self.planner = planner
        self.window = window
        self.min_n = min_n
        self.max_pending = max_pending
        self._pred: Dict[str, Tuple[Hashable, float]] = {}
        self._ratios: "collections.deque[float]" = collections.deque(maxlen=window)
        self._held: List[Tuple[Hashable, float, float]] = []     # (group, predicted, measured) before min_n
        self._lock = threading.Lock()
        self.applied = 0
        self.corrections: Dict[Hashable, float] = collections.defaultdict(float)

    def expect(self, pod_key: str, group: Hashable, predicted_ms: float) -> None:
        if predicted_ms > 0:
            with self._lock:
                self._pred[pod_key] = (group, float(predicted_ms))
                if len(self._pred) > self.max_pending:          # pods never seen to finish
                    self._pred.pop(next(iter(self._pred)))

    def refresh(self, pod_key: str, group: Hashable, predicted_ms: float) -> None:
        """Update a pending pod's prediction (a co-runner joined its group)."""
        with self._lock:
            if pod_key in self._pred and predicted_ms > 0:
                self._pred[pod_key] = (group, float(predicted_ms))

    def forget(self, pod_key: str) -> None:
        with self._lock:
            self._pred.pop(pod_key, None)

    def completed(self, pod: Obj) -> bool:
        """A terminal pod: fold its measured-vs-predicted time into its group's backlog."""
        key = O.key(pod)
        if (pod.get("status") or {}).get("phase") != "Succeeded":
            self.forget(key)                # failed: its time measures nothing
            return False
        ms = measured_ms(pod)
        if ms is None:
            # no measurement YET: the node agent writes busy-ms after it sees the pod terminate
            # (agent.busy), a later update of the same pod; the prediction stays pending until
            # then or until the pod is deleted (forget)
            return False
        with self._lock:
            hit = self._pred.pop(key, None)
        if hit is None:
            return False
        group, pred = hit
        with self._lock:
            self._ratios.append(ms / pred)
            self._held.append((group, pred, ms))
            if len(self._ratios) < self.min_n:
                return True
            med = statistics.median(self._ratios)
            held, self._held = self._held, []
        by: Dict[Hashable, float] = collections.defaultdict(float)
        for g, p, m in held:
            # the planner bounds what one completion can do (planner.observe_time: clipped
            # ratios, a window median per GPU, a clipped relative backlog)
            self.planner.observe_time(g, p, m / med)
            by[g] += m / med - p
        for g, d in by.items():
            self.corrections[g] += d
        self.applied += len(by)
        return True
