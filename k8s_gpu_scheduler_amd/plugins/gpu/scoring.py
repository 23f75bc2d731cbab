"""SLO / interference scoring math (pure, side-effect free).

Re-creates the per-UUID score of the reference's `Logic`
(reference pkg/plugins/gpu_plugin/gpu_plugins.go:558-757, spec in SURVEY.md §2.7.2):

  term(SLO, pred, intf):  violated (SLO > pred - intf): neg  1/(1+(|(SLO-(pred-intf))/SLO|+1)^2)
                          satisfied:                     pos  1/(1+ |(SLO-(pred-intf))/SLO|)
  aggregate: k = n_neg/(n_neg+n_pos); both -> 100((1-k)mean(pos) + k mean(neg));
             only one kind -> 100 mean(kind); none -> 0.

Numerics follow Go exactly: SLO / predictions / interference are float32 and the
interference sum accumulates in float32 (gpu_plugins.go:589-612), the ratio
`(1/SLO)*(SLO-(pred-intf))` is evaluated in float32 then widened, the rest is float64,
and the node score is `int64(tmpScore)` (truncation).  The native C++ core
(`_native/_core`, native/core/score.cpp) implements the same function for batches of
devices; `score_devices` dispatches to it when built.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

f32 = np.float32
# below this many residents the Python loop beats packing arrays for the C++ core
NATIVE_MIN_RESIDENTS = 8


def f32_interference(values: Iterable[float]) -> np.float32:
    acc = f32(0.0)
    for v in values:
        acc = f32(acc + f32(v))
    return acc


def slo_term(slo: float, pred: float, intf: float) -> Tuple[bool, float]:
    """(is_negative, value) for one pod on one device."""
    s, p, i = f32(slo), f32(pred), f32(intf)
    eff = f32(p - i)
    ratio = float(f32(f32(f32(1.0) / s) * f32(s - eff)))
    if s > eff:
        return True, 1.0 / (1.0 + math.pow(abs(ratio) + 1.0, 2))
    return False, 1.0 / (1.0 + abs(ratio))


@dataclass
class TermAcc:
    neg_sum: float = 0.0
    pos_sum: float = 0.0
    n_neg: int = 0
    n_pos: int = 0

    def add(self, slo: float, pred: float, intf: float) -> None:
        neg, v = slo_term(slo, pred, intf)
        if neg:
            self.neg_sum += v
            self.n_neg += 1
        else:
            self.pos_sum += v
            self.n_pos += 1

    def score(self, factor: float = 100.0) -> float:
        if self.n_pos > 0 and self.n_neg > 0:
            k = self.n_neg / (self.n_neg + self.n_pos)
            return factor * ((1 - k) * self.pos_sum / self.n_pos) + factor * (k * self.neg_sum / self.n_neg)
        if self.n_neg > 0:
            return factor * (self.neg_sum / self.n_neg)
        if self.n_pos > 0:
            return factor * (self.pos_sum / self.n_pos)
        return 0.0


def match_column(name: str, table: Dict[str, float]) -> Optional[float]:
    """First interference column that is a substring of name with '-'→'_'
    (reference gpu_plugins.go:600-605,708-712)."""
    nm = name.replace("-", "_")
    for col, val in table.items():
        if col in nm:
            return val
    return None


@dataclass
class Resident:
    name: str
    slo: float
    conf: Dict[str, float] = field(default_factory=dict)     # configuration predictions
    intf: Dict[str, float] = field(default_factory=dict)     # interference row (resident_<model>)
    conf_col: str = ""                                       # column used for pred


def device_score(residents: Sequence[Resident], incoming_name: str, incoming_slo: float,
                 incoming_pred: float, incoming_intf: Dict[str, float], default_col: str) -> float:
    """Score of one device (float; the caller truncates).  `incoming_pred == -1` means
    "no configuration qualifies" (resident terms only), as in gpu_plugins.go:667-696."""
    acc = TermAcc()
    for r in residents:
        if r.slo == 0:
            continue
        col = r.conf_col or default_col
        if col not in r.conf:
            continue
        pred = r.conf[col]
        vals = []
        for c in residents:
            if c.name == r.name or c.name == incoming_name:
                continue
            v = match_column(c.name, r.intf)
            if v is not None:
                vals.append(v)
        v = match_column(incoming_name, r.intf)
        if v is not None:
            vals.append(v)
        acc.add(r.slo, pred, float(f32_interference(vals)))
    if incoming_pred == -1:
        return acc.score()
    vals = []
    for c in residents:
        if c.name == incoming_name:
            continue
        v = match_column(c.name, incoming_intf)
        if v is not None:
            vals.append(v)
    acc.add(incoming_slo, incoming_pred, float(f32_interference(vals)))
    return acc.score()


def pick_mps_config(conf: Dict[str, float], slo: float, model: str = "V100",
                    parts: Sequence[int] = (1, 2, 4)) -> Tuple[str, float]:
    """Smallest predicted throughput that still exceeds the SLO among <p>P_<model>
    (reference gpu_plugins.go:638-651).  Returns (column, pred); pred = -1 if none
    qualifies and the column stays the 1P default."""
    idx, pred = f"1P_{model}", -1.0
    s = float(f32(slo))
    for p in parts:
        col = f"{p}P_{model}"
        v = conf.get(col)
        if v is not None and float(f32(v)) > s and (pred == -1 or float(f32(v)) < pred):
            idx, pred = col, float(f32(v))
    return idx, pred


def reconfigure_choice(conf: Dict[str, float], slo: float, model: str = "A30",
                       fixed: bool = False) -> int:
    """Index into MIG_CONFIGS (0 = all-4g = 1P, 1 = 2P, 2 = 4P).

    parity (reference gpu_plugins.go:365-399): satisfied branch 100/(1+(SLO-pred)) goes
    negative for pred > SLO+1, so with the shipped data the result is always 0
    (SURVEY §2.9 #4).  fixed: most partitions whose prediction still meets the SLO,
    else the configuration with the highest prediction."""
    opts = [1, 2, 4]
    if fixed:
        ok = [i for i, p in enumerate(opts) if conf.get(f"{p}P_{model}", -math.inf) >= slo]
        if ok:
            return max(ok)
        best = max(range(3), key=lambda i: conf.get(f"{opts[i]}P_{model}", -math.inf))
        return best
    best_i, best = 0, 0.0
    s = float(f32(slo))
    for p in opts:
        col = f"{p}P_{model}"
        if col not in conf:
            continue
        pred = float(f32(conf[col]))
        if s > pred:
            sc = 100 / (1 + math.pow(float(f32(f32(s) - f32(pred) + f32(1))), 2))
        else:
            sc = 100 / (1 + float(f32(f32(s) - f32(pred))))
        if sc >= best:
            best = sc
            best_i = p - 1
    if best_i == 3:
        best_i -= 1
    return best_i


def mps_env(value: str) -> Tuple[str, str]:
    """PostBind MPS mapping; checks "2" before "4" (reference gpu_plugins.go:896-903)."""
    if "2" in value:
        return "0=16350MB", "50"
    if "4" in value:
        return "0=8175MB", "25"
    return "", ""


def workload_column(name: str, row: Dict[str, float]) -> Optional[str]:
    """The interference column a pod name resolves to (first column that is a substring of
    the name with '-'→'_', as match_column), or None."""
    nm = name.replace("-", "_")
    for col in row:
        if col in nm:
            return col
    return None


@dataclass
class DeviceSummary:
    """Fixed-mode per-device resident summary, rebuilt only when the device's residents
    change (the ledger invalidates it on Reserve/Unreserve).  Each resident term keeps
    its SLO, its predicted throughput and the interference it already receives from the
    OTHER residents, so scoring an incoming pod is O(residents) dict lookups instead of
    the reference's O(residents^2) substring scans per candidate (gpu_plugins.go:589-612)."""
    terms: List[Tuple[str, float, float, float, Dict[str, float]]]   # name, slo, pred, base intf, intf row
    cols: List[Tuple[str, str]]                                       # (name, interference column)


def build_device_summary(residents: Sequence[Tuple[str, float, Optional[float], Dict[str, float]]]) -> DeviceSummary:
    """residents: (name, slo, pred in its own column or None, its interference row)."""
    cols = []
    for name, _, _, row in residents:
        c = workload_column(name, row) if row else None
        if c is not None:
            cols.append((name, c))
    terms = []
    for name, slo, pred, row in residents:
        if slo == 0 or pred is None:
            continue
        base = 0.0
        for other, c in cols:
            if other != name:
                base += row.get(c, 0.0)
        terms.append((name, float(slo), float(pred), base, row))
    return DeviceSummary(terms, cols)


def fast_device_score(s: DeviceSummary, x_name: str, x_col: Optional[str], x_slo: float, x_pred: float,
                      x_intf: Dict[str, float]) -> float:
    """The device_score objective (same terms and aggregation) in float64 from a
    DeviceSummary -- fixed mode only; parity mode keeps the float32 Go numerics."""
    neg_sum = pos_sum = 0.0
    n_neg = n_pos = 0
    for name, slo, pred, base, row in s.terms:
        i = base
        if x_col is not None and name != x_name:
            i += row.get(x_col, 0.0)
        d = (slo - (pred - i)) / slo
        if d > 0:
            neg_sum += 1.0 / (1.0 + (abs(d) + 1.0) ** 2)
            n_neg += 1
        else:
            pos_sum += 1.0 / (1.0 + abs(d))
            n_pos += 1
    if x_pred != -1 and x_slo > 0:
        i = 0.0
        for other, c in s.cols:
            if other != x_name:
                i += x_intf.get(c, 0.0)
        d = (x_slo - (x_pred - i)) / x_slo
        if d > 0:
            neg_sum += 1.0 / (1.0 + (abs(d) + 1.0) ** 2)
            n_neg += 1
        else:
            pos_sum += 1.0 / (1.0 + abs(d))
            n_pos += 1
    if n_pos and n_neg:
        k = n_neg / (n_neg + n_pos)
        return 100.0 * ((1 - k) * pos_sum / n_pos) + 100.0 * (k * neg_sum / n_neg)
    if n_neg:
        return 100.0 * neg_sum / n_neg
    if n_pos:
        return 100.0 * pos_sum / n_pos
    return 0.0


def score_devices(residents_per_device: List[Sequence[Resident]], incoming_name: str, incoming_slo: float,
                  incoming_pred: float, incoming_intf: Dict[str, float], default_col: str) -> List[float]:
    """Batch form; uses the native core when available (identical results)."""
    try:
        from ..._native import score_core as _core
    except Exception:
        _core = None
    if _core is not None and _core.available() and sum(len(r) for r in residents_per_device) >= NATIVE_MIN_RESIDENTS:
        return _core.score_devices(residents_per_device, incoming_name, incoming_slo, incoming_pred,
                                   incoming_intf, default_col)
    return [device_score(r, incoming_name, incoming_slo, incoming_pred, incoming_intf, default_col)
            for r in residents_per_device]
