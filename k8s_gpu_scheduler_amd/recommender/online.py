"""Pairwise interference learned online from what co-running pods actually achieved.

The reference's interference matrix is measured offline and only re-read when its file
changes (reference pkg/recommender/recom_server.py:74-134, interference_train.ods); its
Score sums the matrix entries of a pod's co-residents to predict the throughput it loses
(gpu_plugins.go:589-612).  Here the same additive model is *fitted* to live observations:
a pod of workload `a` that achieved throughput `t` while sharing a GPU with pods of
workloads `b_1..b_k` lost `loss = predicted_alone(a) - t`, modelled as
`sum_j intf[a][b_j]`.  Each row `a` is a ridge regression over the 18 (or however many)
co-runner columns, shrunk toward the prior (offline / imputed) row, so rows with few
observations keep the measured table and well-observed rows follow the hardware.

Rows see few observations each (a row per workload, ~5 per row in a 20-epoch bench), so
the ridge target is not the prior row itself but the prior row SCALED: a global factor G
(least squares of observed loss on prior-predicted loss over every observation) and a per-row
factor g_a shrunk toward G (`kappa` observations' worth of pull).  A systematic bias of the
pairwise-measured table under 4-way co-run -- it under-predicts what the memory system takes
from co-running pods -- is thus learned from all rows at once, and the per-column ridge
refines what the data supports.  Off by default (`scale=False`: an unseen entry keeps its
prior value exactly); the bench's control plane turns it on (`--online-scale`, default 1:
prequential MAE / prior 0.86-0.90 vs 0.97-0.98 without it at the driver's 20 steps on MI355X,
pods/s unchanged -- profiles/archive/r02_online_scale_ab/).

`prequential` error bookkeeping (predict each observation with the current model before
learning from it) measures whether the online table predicts better than the prior.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence

import numpy as np


class OnlineInterference:
    def __init__(self, labels: Sequence[str], columns: Sequence[str], prior: np.ndarray, lam: float = 4.0,
                 refit_every: int = 32, scale: bool = False, kappa: float = 2.0, scale_bounds=(0.25, 4.0)):
        self.labels, self.columns = list(labels), list(columns)
        w, c = len(self.labels), len(self.columns)
        prior = np.asarray(prior, dtype=np.float64)
        if prior.shape != (w, c):
            raise ValueError(f"prior shape {prior.shape} != ({w}, {c})")
        fill = np.nanmean(prior) if np.isfinite(prior).any() else 0.0
        self.prior = np.where(np.isfinite(prior), prior, fill)
        self.lam = lam
        self.refit_every = refit_every
        self._ata = np.zeros((w, c, c))
        self._atb = np.zeros((w, c))
        self._n = np.zeros(w, dtype=np.int64)
        # prior-scale sufficient statistics per row: sum p*y, sum p*p (p = prior-predicted loss)
        self.scale, self.kappa, self.scale_bounds = scale, kappa, scale_bounds
        self._py = np.zeros(w)
        self._pp = np.zeros(w)
        self.row_scale = np.ones(w)
        self.global_scale = 1.0
        self.matrix = self.prior.copy()
        self.version = 0
        self._pending: List[tuple] = []
        self._lock = threading.Lock()
        self.err = {"prior": 0.0, "online": 0.0, "n": 0}

    def predict_loss(self, a: int, others: Sequence[int], prior: bool = False) -> float:
        row = (self.prior if prior else self.matrix)[a]
        return float(sum(row[b] for b in others))

    def observe(self, a: int, others: Sequence[int], loss: float) -> bool:
        """Learn from one pod; returns True when the matrix was refitted.  Observations are
        queued and folded into the per-row normal equations in one vectorised pass at refit
        time, so the per-pod cost is a few dict/array lookups."""
        if not len(others) or not np.isfinite(loss):
            return False
        pr, on = self.prior[a], self.matrix[a]
        with self._lock:
            self.err["prior"] += abs(sum(pr[b] for b in others) - loss)
            self.err["online"] += abs(sum(on[b] for b in others) - loss)
            self.err["n"] += 1
            self._pending.append((a, tuple(others), loss))
            if len(self._pending) >= self.refit_every:
                self._refit()
                return True
        return False

    def _fold(self) -> None:
        if not self._pending:
            return
        n, c = len(self._pending), len(self.columns)
        rows = np.fromiter((p[0] for p in self._pending), dtype=np.int64, count=n)
        y = np.fromiter((p[2] for p in self._pending), dtype=np.float64, count=n)
        x = np.zeros((n, c))
        for i, (_, others, _) in enumerate(self._pending):
            for b in others:
                x[i, b] += 1.0
        for a in np.unique(rows):
            sel = rows == a
            xa = x[sel]
            self._ata[a] += xa.T @ xa
            self._atb[a] += xa.T @ y[sel]
            self._n[a] += int(sel.sum())
            pa = xa @ self.prior[a]
            self._py[a] += float(pa @ y[sel])
            self._pp[a] += float(pa @ pa)
        self._pending.clear()

    def _refit(self) -> None:
        self._fold()
        eye = np.eye(len(self.columns))
        m = self.matrix.copy()
        lo, hi = self.scale_bounds
        if self.scale and self._pp.sum() > 0:
            G = float(np.clip(self._py.sum() / self._pp.sum(), lo, hi))
            seen = self._n > 0
            k = self.kappa * float(self._pp[seen].sum() / max(1, int(self._n[seen].sum())))
            self.global_scale = G
            self.row_scale = np.where(seen, np.clip((self._py + k * G) / (self._pp + k + 1e-30), lo, hi), G)
            m = self.prior * self.row_scale[:, None]       # unseen rows follow the global scale
        for a in np.nonzero(self._n)[0]:
            lhs = self._ata[a] + self.lam * eye
            rhs = self._atb[a] + self.lam * self.prior[a] * (self.row_scale[a] if self.scale else 1.0)
            m[a] = np.maximum(np.linalg.solve(lhs, rhs), 0.0)    # a co-runner never adds throughput
        self.matrix = m
        self.version += 1

    def refit(self) -> None:
        with self._lock:
            self._refit()

    def mae(self) -> Dict[str, Optional[float]]:
        n = self.err["n"]
        return {"n": n, "prior": self.err["prior"] / n if n else None,
                "online": self.err["online"] / n if n else None}

    def rows(self) -> List[List[float]]:
        return self.matrix.tolist()
