"""Request right-sizing from profiler history (BASELINE config 5: "recommender loop:
resize 16 pods' GPU requests from profiler/Redis history under Poisson arrivals").

The reference has no resize path (its recommender only imputes).
Policy, per pod (history = samples the node agent appended to `gpusched:hist:<pod>`):

* HBM: p95 of observed `hbm_gib` x (1 + headroom), rounded up to `hbm_quantum_gib`,
  never below `min_hbm_gib`.
* CUs: the smallest partition share s in {32, 64, 128, 256} whose throughput
  (measured at that share if sampled, else scaled from the configuration predictions
  `<P>P_MI355X`, else from the observed throughput x share ratio; observed throughput
  = its `tput_quantile` quantile) still meets
  SLO x (1 + slo_margin).  No SLO -> keep p95 CU-busy x allotment, rounded to a share.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, Dict, List, Optional

SHARES = (32, 64, 128, 256)
SHARE_TO_P = {256: 1, 128: 2, 64: 4, 32: 8}


@dataclass
class ResizeAdvice:
    cu: int
    hbm_gib: float
    samples: int
    reason: str


def _pct(xs: List[float], q: float) -> float:
    if not xs:
        return 0.0
    s = sorted(xs)
    i = min(len(s) - 1, max(0, int(math.ceil(q * len(s))) - 1))
    return s[i]


def recommend(history: List[Dict[str, Any]], requested_cu: int, requested_hbm_gib: float, slo: float = 0.0,
              conf_predictions: Optional[Dict[str, float]] = None, model: str = "MI355X",
              headroom: float = 0.15, slo_margin: float = 0.05, hbm_quantum_gib: float = 1.0,
              min_hbm_gib: float = 1.0, min_samples: int = 3, tput_quantile: float = 0.25) -> ResizeAdvice:
    """tput_quantile: which quantile of the throughputs observed at a share counts as that
    share's throughput -- below the median, so a share is only picked when most of its
    observed runs (under whatever co-runners they had) met the SLO."""
    if len(history) < min_samples:
        return ResizeAdvice(requested_cu, requested_hbm_gib, len(history), "insufficient history")
    hbm = [float(h.get("hbm_gib", 0.0)) for h in history]
    hbm_rec = max(min_hbm_gib, math.ceil(_pct(hbm, 0.95) * (1 + headroom) / hbm_quantum_gib) * hbm_quantum_gib)
    # throughput observed per share
    by_share: Dict[int, List[float]] = {}
    for h in history:
        if "throughput" in h and h.get("cu"):
            by_share.setdefault(int(h["cu"]), []).append(float(h["throughput"]))
    need = slo * (1 + slo_margin)
    if slo > 0:
        def tput(share: int) -> Optional[float]:
            if share in by_share:
                return _pct(by_share[share], tput_quantile)
            if conf_predictions:
                v = conf_predictions.get(f"{SHARE_TO_P[share]}P_{model}")
                if v is not None and v > 0:
                    return v
            if by_share:
                # sub-linear extrapolation from the nearest observed share
                s0 = min(by_share, key=lambda s: abs(math.log2(s / share)))
                t0 = _pct(by_share[s0], tput_quantile)
                return t0 * (share / s0) ** 0.85
            return None
        for s in SHARES:
            t = tput(s)
            if t is not None and t >= need:
                return ResizeAdvice(s, hbm_rec, len(history), f"smallest share meeting SLO {slo:g}: {t:.1f}")
        return ResizeAdvice(256, hbm_rec, len(history), "no share meets SLO; full GPU")
    busy = [float(h.get("cu_busy", 1.0)) for h in history]
    eff = _pct(busy, 0.95) * max(requested_cu, 1) * (1 + headroom)
    cu = next((s for s in SHARES if s >= eff), 256)
    return ResizeAdvice(cu, hbm_rec, len(history), "p95 CU busy")
