"""Observed per-workload GPU cost, learned from what pods actually consumed.

The recommender's configuration matrix predicts a workload's throughput when it runs
ALONE on a share of a GPU (reference pkg/recommender/recommender/configurations_train.ods:
`<N>P_<MODEL>` columns).  A Burstable pod co-running with others on a whole MI355X costs
something different: small GEMMs that cannot fill the chip alone are cheap in a mix, HBM
streams are not.  The executors report, per finished pod, the CU-share-time it held
(elapsed ms x its units / units per GPU -- the share of the GPU's busy time attributable
to it) per iteration; this model keeps an exponentially weighted mean per workload, and
the GPU plugin uses it (when present) instead of 1/throughput for the pod's predicted
GPU time -- the profiler-history -> scheduler loop of the MI355X design (BASELINE.json
north star: "the profiler sidecar samples ... per pod into Redis and the recommender
resizes GPU requests from that history").

Workload identity follows the recommender's rule: the first known workload label that is
a substring of the pod name with '-' -> '_' (reference recom_server.py:67-71).
"""
from __future__ import annotations

import threading
from typing import Dict, Iterable, Optional, Tuple


class WorkCostModel:
    def __init__(self, alpha: float = 0.2, min_samples: int = 1):
        self.alpha = alpha
        self.min_samples = min_samples
        self._lock = threading.Lock()
        self._cost: Dict[str, Tuple[float, int]] = {}      # label -> (ewma seconds/iter, samples)
        self._labels: Tuple[str, ...] = ()
        self._resolve: Dict[str, Optional[str]] = {}
        self.version = 0

    def observe(self, label: str, seconds_per_iter: float, weight: int = 1) -> None:
        """One observation (or `weight` pods' mean) of a workload's per-iteration cost."""
        if seconds_per_iter <= 0 or weight <= 0:
            return
        with self._lock:
            cur = self._cost.get(label)
            if cur is None:
                self._cost[label] = (seconds_per_iter, weight)
                # longest labels first, so 'x_4096' is not shadowed by a shorter prefix
                self._labels = tuple(sorted(self._cost, key=len, reverse=True))
                self._resolve.clear()
            else:
                a = 1.0 - (1.0 - self.alpha) ** weight
                self._cost[label] = (cur[0] + a * (seconds_per_iter - cur[0]), cur[1] + weight)
            self.version += 1

    def observe_many(self, rows: Iterable[Tuple[str, float, int]]) -> None:
        for label, s, n in rows:
            self.observe(label, s, n)

    def label_for(self, pod_name: str) -> Optional[str]:
        hit = self._resolve.get(pod_name, False)
        if hit is not False:
            return hit
        nm = pod_name.replace("-", "_")
        lab = next((lb for lb in self._labels if lb in nm), None)
        if len(self._resolve) > 65536:
            self._resolve.clear()
        self._resolve[pod_name] = lab
        return lab

    def seconds_per_iter(self, pod_name: str) -> Optional[float]:
        lab = self.label_for(pod_name)
        if lab is None:
            return None
        v = self._cost.get(lab)
        if v is None or v[1] < self.min_samples:
            return None
        return v[0]

    def snapshot(self) -> Dict[str, float]:
        with self._lock:
            return {k: v[0] for k, v in self._cost.items()}
