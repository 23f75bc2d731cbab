"""Matrix-completion models behind the recommender.

* `IterativeImputerModel` -- the reference's model, `IterativeImputer(max_iter=10,
  random_state=0)` fitted on the user x item matrix, `predict` = `transform`
  (reference pkg/recommender/recommender/recommender.py:11-27).  Used in parity mode.
* `SVDImputer` -- iterative truncated-SVD completion with k latent factors; re-creates
  the capability of the reference's orphaned `SVDRecommender`
  (reference pkg/recommender/recommender/__pycache__/SVD.cpython-38.pyc, source absent;
  SURVEY.md §0 "Orphans": k latent factors).
* `ALSImputer` -- alternating least squares in PyTorch.  Runs on the MI355X (HIP device
  tensors; the per-row normal-equation solves are batched `torch.linalg.solve`) for the
  large usage-history matrices the profiler accumulates (pods x configurations), and on
  CPU otherwise.

All share: `fit(X)` with NaN = missing, `predict(rows)` returning completed rows where
observed entries are kept and missing entries are imputed.
"""
from __future__ import annotations

from typing import Optional

import numpy as np


class ImputerBase:
    name = "base"

    def fit(self, X: np.ndarray) -> "ImputerBase":
        raise NotImplementedError

    def predict(self, rows: np.ndarray) -> np.ndarray:
        raise NotImplementedError


class IterativeImputerModel(ImputerBase):
    name = "iterative"

    def __init__(self, max_iter: int = 10, random_state: int = 0):
        self.max_iter, self.random_state = max_iter, random_state
        self.imp = None

    def fit(self, X: np.ndarray) -> "IterativeImputerModel":
        from sklearn.experimental import enable_iterative_imputer  # noqa: F401
        from sklearn.impute import IterativeImputer
        imp = IterativeImputer(max_iter=self.max_iter, random_state=self.random_state)
        imp.fit(np.asarray(X, dtype=float))
        self.imp = imp
        return self

    def predict(self, rows: np.ndarray) -> np.ndarray:
        return np.asarray(self.imp.transform(np.asarray(rows, dtype=float)))


class SVDImputer(ImputerBase):
    """Soft-impute style: fill missing with column means, then repeat
    X_hat = U_k S_k V_k^T on the filled matrix, re-imposing observed entries."""
    name = "svd"

    def __init__(self, k: int = 4, iters: int = 100, tol: float = 1e-6):
        self.k, self.iters, self.tol = k, iters, tol
        self.mean_: Optional[np.ndarray] = None
        self.std_: Optional[np.ndarray] = None
        self.V_: Optional[np.ndarray] = None

    def fit(self, X: np.ndarray) -> "SVDImputer":
        X = np.asarray(X, dtype=float)
        mask = ~np.isnan(X)
        mean = np.nanmean(np.where(mask, X, np.nan), axis=0)
        mean = np.where(np.isnan(mean), 0.0, mean)
        std = np.nanstd(np.where(mask, X, np.nan), axis=0)
        std = np.where((std == 0) | np.isnan(std), 1.0, std)
        Z = np.where(mask, (X - mean) / std, 0.0)
        k = max(1, min(self.k, min(Z.shape) - 1 if min(Z.shape) > 1 else 1))
        prev = None
        for _ in range(self.iters):
            U, S, Vt = np.linalg.svd(Z, full_matrices=False)
            L = (U[:, :k] * S[:k]) @ Vt[:k]
            Znew = np.where(mask, Z, L)
            if prev is not None and np.linalg.norm(Znew - prev) <= self.tol * (np.linalg.norm(prev) + 1e-12):
                Z = Znew
                break
            prev, Z = Z, Znew
        _, _, Vt = np.linalg.svd(Z, full_matrices=False)
        self.mean_, self.std_, self.V_ = mean, std, Vt[:k].T
        return self

    def predict(self, rows: np.ndarray) -> np.ndarray:
        rows = np.asarray(rows, dtype=float)
        out = rows.copy()
        V = self.V_
        for i, r in enumerate(rows):
            m = ~np.isnan(r)
            z = np.where(m, (r - self.mean_) / self.std_, 0.0)
            if m.any():
                # least squares for the latent code from the observed coordinates only
                coef, *_ = np.linalg.lstsq(V[m], z[m], rcond=None)
                zhat = V @ coef
            else:
                zhat = np.zeros_like(z)
            out[i] = np.where(m, r, zhat * self.std_ + self.mean_)
        return out


class ALSImputer(ImputerBase):
    """Regularised ALS on standardised data, in torch (device = "cuda" runs on the GPU)."""
    name = "als"

    def __init__(self, k: int = 4, iters: int = 30, reg: float = 0.05, device: str = "cpu", seed: int = 0):
        self.k, self.iters, self.reg, self.device, self.seed = k, iters, reg, device, seed
        self.mean_ = self.std_ = None
        self.V_ = None

    def fit(self, X: np.ndarray) -> "ALSImputer":
        import torch
        X = np.asarray(X, dtype=np.float64)
        mask = ~np.isnan(X)
        mean = np.nanmean(np.where(mask, X, np.nan), axis=0)
        mean = np.where(np.isnan(mean), 0.0, mean)
        std = np.nanstd(np.where(mask, X, np.nan), axis=0)
        std = np.where((std == 0) | np.isnan(std), 1.0, std)
        dev = torch.device(self.device)
        Z = torch.tensor(np.where(mask, (X - mean) / std, 0.0), dtype=torch.float32, device=dev)
        M = torch.tensor(mask, dtype=torch.float32, device=dev)
        g = torch.Generator(device="cpu").manual_seed(self.seed)
        n, m = Z.shape
        k = max(1, min(self.k, m))
        U = (0.1 * torch.randn(n, k, generator=g)).to(dev)
        V = (0.1 * torch.randn(m, k, generator=g)).to(dev)
        eye = torch.eye(k, device=dev) * self.reg
        for _ in range(self.iters):
            # rows: (V^T diag(M_i) V + reg I) u_i = V^T (M_i * z_i)   -- batched solves
            A = torch.einsum("ij,jk,jl->ikl", M, V, V) + eye
            b = (M * Z) @ V
            U = torch.linalg.solve(A, b.unsqueeze(-1)).squeeze(-1)
            A = torch.einsum("ij,ik,il->jkl", M, U, U) + eye
            b = (M * Z).T @ U
            V = torch.linalg.solve(A, b.unsqueeze(-1)).squeeze(-1)
        self.mean_, self.std_ = mean, std
        self.V_ = V.detach().cpu().double().numpy()
        return self

    def predict(self, rows: np.ndarray) -> np.ndarray:
        rows = np.asarray(rows, dtype=float)
        out = rows.copy()
        V = self.V_
        k = V.shape[1]
        for i, r in enumerate(rows):
            m = ~np.isnan(r)
            z = np.where(m, (r - self.mean_) / self.std_, 0.0)
            Vm = V[m]
            u = np.linalg.solve(Vm.T @ Vm + self.reg * np.eye(k), Vm.T @ z[m]) if m.any() else np.zeros(k)
            out[i] = np.where(m, r, (V @ u) * self.std_ + self.mean_)
        return out


MODELS = {"iterative": IterativeImputerModel, "svd": SVDImputer, "als": ALSImputer}


def make_imputer(kind: str = "iterative", **kw) -> ImputerBase:
    if kind not in MODELS:
        raise KeyError(f"unknown imputer {kind!r}; have {sorted(MODELS)}")
    return MODELS[kind](**kw)
