"""Cold start of the co-run model for a workload it has never seen co-run.

The co-run model (models.corun) has one row per workload: its alone time and its fluid-model
sensitivity / pressure vectors u, v, fitted on measured co-run groups.  A new workload has
none of those groups, so `CorunModel.wid` returned -1 for it, the burst planner dropped its
pods and Score fell back to the pairwise table (which does not know it either).

The reference's recommender exists to complete partially observed rows (reference
pkg/recommender/recommender/recommender.py:11-27: SVD / iterative imputation of the
configuration and interference matrices; recom_server.py:155-164 serves the completed
rows).  Here the partially observed row is the new workload's ALONE profile -- which the node
agent already collects: a webhook-profiled pod that ran alone on its device is a 1-pod co-run
observation (agent.corun_observer), its kernel trace gives the time per iteration and its
kernel mix the MFMA share of its busy time (agent.pod_profiler.summarize_kernel_stats; the
PMC pass's MFMA counters when present).  From that:

  * alone_ms  = measured ms per iteration (Burstable, alone on the GPU: the model's unit);
  * u, v      = the geometric kernel-weighted mean of the catalog rows nearest in
                (MFMA share, log alone time): the resource shape decides how a workload
                presses on and suffers from others, its length how much the short-kernel
                launch overheads of co-running hurt it.

Online observations then refine the row like every other (models.corun.OnlineCorun: its
alone-time scale from the groups it co-runs in).

Leave-one-workload-out on the MI355X co-run groups (tools/corun_coldstart_eval.py,
profiles/r04_coldstart/loo.json): the model refitted WITHOUT workload X, X cold-started from
its alone groups only -- X's co-run throughput is predicted within a mean 5.8 % (median 5.0,
worst 10.1), against 4.8 % held-out error of those fits on the workloads they saw (1.2x),
4.6 % for X's own fitted row and 16.7 % for the roofline prior row.
"""
from __future__ import annotations

from typing import Any, Optional, Sequence, Tuple

import numpy as np

# feature scales of the neighbour distance: MFMA share (0..1) and log alone ms
SCALE_MFMA = 0.2
SCALE_LOG_ALONE = 0.5
NEIGHBOURS = 3


def mfma_share(name: str) -> Optional[float]:
    """Roofline MFMA share of a catalog workload's alone time (None if unknown)."""
    from . import workloads as W
    rf = W.roofline_split(name.replace("_", "-"))
    if not rf:
        return None
    m, h = rf
    return float(m / max(m + h, 1e-30))


def catalog_features(model: Any) -> np.ndarray:
    """[n, 2] (MFMA share, log alone ms) of the model's rows (share 0.5 when unknown)."""
    out = np.zeros((len(model.names), 2))
    for i, n in enumerate(model.names):
        s = model.meta.get("mfma_share", {}).get(n) if isinstance(model.meta.get("mfma_share"), dict) else None
        if s is None:
            s = mfma_share(n)
        out[i, 0] = 0.5 if s is None else s
        out[i, 1] = np.log(max(float(model.alone_ms[i]), 1e-9))
    return out


def impute_row(model: Any, alone_ms: float, mfma: Optional[float], exclude: Sequence[int] = (),
               k: int = NEIGHBOURS) -> Tuple[np.ndarray, np.ndarray, list]:
    """(u, v, neighbour names) for a workload with this alone profile.  Without an MFMA share
    the neighbours are picked on the alone time alone."""
    f = catalog_features(model)
    d2 = ((f[:, 1] - np.log(max(alone_ms, 1e-9))) / SCALE_LOG_ALONE) ** 2
    if mfma is not None:
        d2 = d2 + ((f[:, 0] - float(mfma)) / SCALE_MFMA) ** 2
    d = np.sqrt(d2)
    d[list(exclude)] = np.inf
    order = [i for i in np.argsort(d) if np.isfinite(d[i])][:k]
    if not order:
        raise ValueError("cold start: no catalog rows to impute from")
    w = 1.0 / (d[order] + 0.05)
    lu = np.log(np.maximum(model.u[order], 1e-6))
    lv = np.log(np.maximum(model.v[order], 1e-6))
    u = np.exp((w[:, None] * lu).sum(0) / w.sum())
    v = np.exp((w[:, None] * lv).sum(0) / w.sum())
    return u, v, [model.names[i] for i in order]


def with_workload(model: Any, name: str, alone_ms: float, mfma: Optional[float] = None,
                  version: Optional[str] = None) -> Any:
    """A copy of `model` with a cold-started row for `name` (replaced if present)."""
    from .corun import CorunModel
    idx = model.index.get(name)
    excl = [idx] if idx is not None else []
    u, v, nn = impute_row(model, alone_ms, mfma, exclude=excl)
    names = list(model.names)
    A, U, V = model.alone_ms.copy(), model.u.copy(), model.v.copy()
    if idx is None:
        names.append(name)
        A = np.append(A, alone_ms)
        U = np.vstack([U, u])
        V = np.vstack([V, v])
    else:
        A[idx], U[idx], V[idx] = alone_ms, u, v
    meta = dict(model.meta)
    cold = dict(meta.get("cold_start") or {})
    cold[name] = {"alone_ms": round(float(alone_ms), 6), "mfma_share": None if mfma is None else round(float(mfma), 4),
                  "neighbours": nn}
    meta["cold_start"] = cold
    shares = dict(meta.get("mfma_share") or {})
    if mfma is not None:
        shares[name] = float(mfma)
    meta["mfma_share"] = shares
    meta["version"] = version or f"{model.version}+cold-{len(cold)}"
    return CorunModel(names, A, U, V, meta)
