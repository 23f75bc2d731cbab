"""Refit the co-run model on data collected under the current kernels and compare it with the
shipped one (round 6: the 4-wave co-run GEMM changed how pods co-run).

    python tools/corun_refit_eval.py --groups G.json --train-traces T0.json T1.json \
        --heldout-traces T2.json --out NEW.json [--summary S.json]

Isolated groups (`models.corun collect`) plus bench pipeline traces (GPUSCHED_BENCH_TRACE,
`models.corun.timeline_groups`) train the new model (`models.corun.fit`, its own 20 % hold-out of
the multi-pod groups); both models are then scored by mean |log(predicted / measured)| duration
on the held-out seed's timeline groups and on every multi-pod isolated group (the old model never
saw these, the new one saw 80 % of them: its fit report's `test` is the fair isolated number).
"""
from __future__ import annotations

import argparse
import gzip
import json
import os
import sys
from typing import Any, Dict, List

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from k8s_gpu_scheduler_amd.models import corun as C  # noqa: E402


def _load(path: str) -> Any:
    op = gzip.open if path.endswith(".gz") else open
    with op(path, "rt") as f:
        return json.load(f)


def timeline(paths: List[str]) -> List[Dict[str, Any]]:
    out: List[Dict[str, Any]] = []
    for p in paths:
        out += C.timeline_groups(_load(p)["pods"])
    return out


def score(model: C.CorunModel, groups: List[Dict[str, Any]]) -> Dict[str, float]:
    """Mean |log error| of predicted durations over the target members, and the share within 15 %."""
    multi = [d for d in groups if len(d["w"]) >= 2]
    K = max(len(d["w"]) for d in multi)
    wids, iters, mask, ms, st = C.pack_groups(multi, model.names, K)
    tg = C.pack_targets(multi, K)
    pin = np.where(mask & ~tg & (ms > 0), ms + st, 0.0)
    t = model.batch_times(wids, iters, mask, st, pin) - st
    sel = mask & tg
    err = np.abs(np.log(np.maximum(t, 1e-9) / np.maximum(ms, 1e-9)))[sel]
    return {"groups": len(multi), "pods": int(sel.sum()), "mean_abs_log": round(float(err.mean()), 4),
            "within_15pct": round(float(np.mean(err <= np.log(1.15))), 4)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", required=True)
    ap.add_argument("--train-traces", nargs="*", default=[])
    ap.add_argument("--heldout-traces", nargs="*", default=[])
    ap.add_argument("--out", required=True)
    ap.add_argument("--summary", default="")
    ap.add_argument("--ridge", type=float, default=0.05)
    a = ap.parse_args()
    iso = _load(a.groups)["groups"]
    train_tl = timeline(a.train_traces)
    held_tl = timeline(a.heldout_traces)
    new, rep = C.fit(iso + train_tl, ridge=a.ridge)
    new.meta["training_data"] = (f"{os.path.basename(a.groups)} ({len(iso)} isolated 1-4 pod groups) + "
                                 f"{len(train_tl)} pipeline timeline groups of "
                                 f"{', '.join(os.path.basename(p) for p in a.train_traces)}")
    new.save(a.out)
    old = C.CorunModel.load()
    out = {"fit_report": rep,
           "heldout_timelines": {"old": score(old, held_tl), "new": score(new, held_tl)} if held_tl else None,
           "isolated_all": {"old": score(old, iso), "new_seen_80pct": score(new, iso)},
           "train_timelines": {"old": score(old, train_tl), "new": score(new, train_tl)} if train_tl else None,
           "old_version": old.meta.get("version"), "new_version": new.meta.get("version")}
    print(json.dumps(out, indent=1))
    if a.summary:
        with open(a.summary, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
