"""Imputation quality helpers (the reference's recommender/utils.py keeps a distance
matrix / masked mean-error printer and a timer formatter,
reference pkg/recommender/utils.py:45-58, pkg/recommender/recommender/utils.py:4-13)."""
from __future__ import annotations

import numpy as np


def distance_matrix(mask: np.ndarray, target: np.ndarray, predicted: np.ndarray) -> np.ndarray:
    return np.abs(target * mask - predicted * mask)


def masked_mean_error(test_set: np.ndarray, target: np.ndarray, predicted: np.ndarray) -> float:
    """Mean |target - predicted| over the entries that were missing in `test_set`."""
    miss = np.isnan(np.asarray(test_set, dtype=float))
    if not miss.any():
        return 0.0
    return float(np.mean(np.abs(np.asarray(target)[miss] - np.asarray(predicted)[miss])))


def holdout_score(model_factory, X: np.ndarray, frac: float = 0.1, seed: int = 0) -> float:
    """Hide `frac` of the observed entries, fit, and return the masked mean error."""
    rng = np.random.default_rng(seed)
    X = np.asarray(X, dtype=float)
    obs = ~np.isnan(X)
    hide = obs & (rng.random(X.shape) < frac)
    train = X.copy()
    train[hide] = np.nan
    pred = model_factory().fit(train).predict(train)
    return float(np.mean(np.abs(pred[hide] - X[hide]))) if hide.any() else 0.0


def read_timer(seconds: float) -> str:
    minutes = int(seconds // 60)
    hours = int(minutes // 60)
    return f"Elapsed Time: {hours} hours, {minutes % 60} minutes and {int(seconds % 60)} seconds."
