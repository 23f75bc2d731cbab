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

  * CU fill  = the time-weighted fraction of the chip its kernels occupy alone (workgroups /
                CUs; the kernel trace's grid sizes, models.workloads.cu_fill for known mixes).
                The neighbours' u, v are scaled by (fill / neighbours' fill) ** beta: a pod that
                fills the chip alone has no idle CUs to give co-runners, so it presses on them
                and suffers from them more than a neighbour of the same MFMA share and length
                whose kernels leave CUs idle.  beta (sensitivity, pressure) is fitted on the
                model's own rows by leave-one-out: each row imputed from the others, the log
                ratio of its fitted to imputed mean sensitivity / pressure regressed on its log
                fill ratio (fill_betas; ~0.3 / ~0.75 on the MI355X fit, correlation 0.55 / 0.66).

Online observations then refine the row like every other (models.corun.OnlineCorun: its
alone-time scale from the groups it co-runs in).

Workloads outside the catalog's kernel mix (models.workloads.EXTRA, measured on MI355X by
tools/corun_extra_groups.py, scored by tools/corun_extra_eval.py -> profiles/r05_coldstart/):
an fp8-GEMM LLM-like workload whose 512-workgroup GEMMs fill the chip (every catalog GEMM
leaves 40-75 % of the CUs idle at a pod's 64-CU tile budget) and a triad-only one.

Leave-one-workload-out on the MI355X co-run groups (tools/corun_coldstart_eval.py,
profiles/archive/r04_coldstart/loo.json): the model refitted WITHOUT workload X, X cold-started from
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


def cu_fill(name: str) -> Optional[float]:
    """CU fill of a known workload (catalog or extra) at a pod's tile budget, None if unknown."""
    from . import workloads as W
    try:
        return W.cu_fill(W.get(name))
    except KeyError:
        return None


def catalog_fills(model: Any) -> np.ndarray:
    """[n] CU fill of the model's rows (meta "cu_fill", else the known kernel mix; nan unknown)."""
    meta = model.meta.get("cu_fill") if isinstance(model.meta.get("cu_fill"), dict) else {}
    out = np.full(len(model.names), np.nan)
    for i, n in enumerate(model.names):
        f = meta.get(n)
        if f is None:
            f = cu_fill(n)
        if f is not None and f > 0:
            out[i] = float(f)
    return out


_BETAS: dict = {}


def fill_betas(model: Any) -> Optional[Tuple[float, float]]:
    """(beta_sensitivity, beta_pressure): leave-one-out regression of each row's fitted / imputed
    mean sensitivity and pressure (log ratios) on its fill / neighbours' fill (log ratio), through
    the origin, over the rows with a known fill; None with fewer than 6 such rows or no spread."""
    key = (model.version, tuple(model.names))
    if key in _BETAS:
        return _BETAS[key]
    if len(_BETAS) >= 64:                # a long-running recommender refits many versions
        _BETAS.clear()
    F = catalog_fills(model)
    Cm = model.u @ model.v.T
    n = len(model.names)
    feats = catalog_features(model)
    xs, ys, yp = [], [], []
    for i in range(n):
        if not np.isfinite(F[i]) or float(model.alone_ms[i]) <= 0:
            continue
        u, v, nn = impute_row(model, float(model.alone_ms[i]), float(feats[i, 0]), exclude=[i])
        idx = [model.index[x] for x in nn]
        fn = F[idx]
        if not np.all(np.isfinite(fn)):
            continue
        others = [j for j in range(n) if j != i]
        sens_fit, sens_imp = Cm[i, others].mean(), (u @ model.v[others].T).mean()
        pr_fit, pr_imp = Cm[others, i].mean(), (model.u[others] @ v).mean()
        if min(sens_fit, sens_imp, pr_fit, pr_imp) <= 0:
            continue
        xs.append(np.log(F[i] / np.exp(np.log(fn).mean())))
        ys.append(np.log(sens_fit / sens_imp))
        yp.append(np.log(pr_fit / pr_imp))
    out = None
    x = np.asarray(xs)
    if len(x) >= 6 and float(x @ x) > 1e-3:
        out = (float(x @ np.asarray(ys) / (x @ x)), float(x @ np.asarray(yp) / (x @ x)))
    _BETAS[key] = out
    return out


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
               k: int = NEIGHBOURS, fill: Optional[float] = None) -> Tuple[np.ndarray, np.ndarray, list]:
    """(u, v, neighbour names) for a workload with this alone profile.  Without an MFMA share
    the neighbours are picked on the alone time alone; with a CU fill (and fill_betas fitted)
    u, v are scaled by the fill ratio to the neighbours."""
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
    if fill is not None and fill > 0:
        fn = catalog_fills(model)[order]
        betas = fill_betas(model) if np.all(np.isfinite(fn)) else None
        if betas is not None:
            r = float(fill) / float(np.exp((w * np.log(fn)).sum() / w.sum()))
            u = u * r ** betas[0]
            v = v * r ** betas[1]
    return u, v, [model.names[i] for i in order]


def with_workload(model: Any, name: str, alone_ms: float, mfma: Optional[float] = None,
                  version: Optional[str] = None, fill: Optional[float] = None) -> Any:
    """A copy of `model` with a cold-started row for `name` (replaced if present)."""
    from .corun import CorunModel
    idx = model.index.get(name)
    excl = [idx] if idx is not None else []
    u, v, nn = impute_row(model, alone_ms, mfma, exclude=excl, fill=fill)
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
                  "cu_fill": None if fill is None else round(float(fill), 4), "neighbours": nn}
    meta["cold_start"] = cold
    shares = dict(meta.get("mfma_share") or {})
    if mfma is not None:
        shares[name] = float(mfma)
    meta["mfma_share"] = shares
    if fill is not None:
        fills = dict(meta.get("cu_fill") or {})
        fills[name] = float(fill)
        meta["cu_fill"] = fills
    meta["version"] = version or f"{model.version}+cold-{len(cold)}"
    return CorunModel(names, A, U, V, meta)
