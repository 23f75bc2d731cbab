"""Python face of the native scoring core (`_core`): packs residents into flat arrays and
calls `slo_scores` (see native/core/score.cpp)."""
from __future__ import annotations

from typing import Dict, List, Sequence

import numpy as np

from . import core as _load_core  # loader function (package __init__)


def available() -> bool:
    return _load_core() is not None


def score_devices(residents_per_device: List[Sequence], incoming_name: str, incoming_slo: float,
                  incoming_pred: float, incoming_intf: Dict[str, float], default_col: str) -> List[float]:
    from ..plugins.gpu.scoring import f32_interference, match_column
    m = _load_core()
    offsets = [0]
    slo, pred, intf = [], [], []
    inc_pred, inc_intf = [], []
    for residents in residents_per_device:
        for r in residents:
            col = r.conf_col or default_col
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
            slo.append(r.slo)
            pred.append(r.conf[col] if col in r.conf else np.nan)
            intf.append(float(f32_interference(vals)))
        offsets.append(len(slo))
        vals = []
        for c in residents:
            if c.name == incoming_name:
                continue
            v = match_column(c.name, incoming_intf)
            if v is not None:
                vals.append(v)
        inc_pred.append(incoming_pred)
        inc_intf.append(float(f32_interference(vals)))
    out = m.slo_scores(np.asarray(offsets, np.int64), np.asarray(slo, np.float32), np.asarray(pred, np.float32),
                       np.asarray(intf, np.float32), np.float32(incoming_slo), np.asarray(inc_pred, np.float32),
                       np.asarray(inc_intf, np.float32))
    return [float(x) for x in out]
