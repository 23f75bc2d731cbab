"""Cold-start score of the co-run model on workloads outside the catalog.

Input: tools/corun_extra_groups.py's MI355X groups.  For each extra workload X
(models.workloads.EXTRA): X gets a cold-started row (models.coldstart.with_workload) from the
median ms per iteration of its ALONE groups and its roofline MFMA share -- nothing from its
co-run groups -- and the model predicts every multi-pod group containing X.  Reported per X:
the throughput error of X's pods, and of the catalog pods in the same groups (rows fitted on
other boxes' groups: the model's error on this box for workloads it knows).  Both with the
model's catalog alone times as fitted, and with them replaced by this box's alone medians (what
the online learner's alone-time scale converges to).  The bar is the fitted model's held-out
MAE (profiles/archive/r04_coldstart/loo.json: mean of the leave-one-out fits' held-out errors).

    python tools/corun_extra_eval.py gpurun_out/corun_extra_groups.json [--out profiles/r05_coldstart/extra.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def errors(model, groups, sel_fn):
    from k8s_gpu_scheduler_amd.models.corun import pack_groups
    names = model.names
    wids, iters, mask, ms, st = pack_groups(groups, names, 4)
    t = model.batch_times(wids, iters, mask, st) - st
    sel = mask & sel_fn(wids)
    if not sel.any():
        return None
    tp, tm = iters / np.maximum(t, 1e-9) * 1e3, iters / np.maximum(ms, 1e-9) * 1e3
    return {"mae_pct": round(float(100 * np.abs(tp - tm)[sel].mean() / tm[sel].mean()), 3),
            "median_abs_pct": round(float(100 * np.median(np.abs(tp - tm)[sel] / tm[sel])), 3),
            "bias_pct": round(float(100 * (tp - tm)[sel].mean() / tm[sel].mean()), 3),
            "pods": int(sel.sum())}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("groups")
    ap.add_argument("--loo", default=os.path.join(ROOT, "profiles", "archive", "r04_coldstart", "loo.json"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_coldstart", "extra.json"))
    a = ap.parse_args(argv)
    from k8s_gpu_scheduler_amd.models.coldstart import cu_fill, fill_betas, mfma_share, with_workload
    from k8s_gpu_scheduler_amd.models.corun import CorunModel
    d = json.load(open(a.groups))
    groups, extra = d["groups"], d["extra"]
    held_out = json.load(open(a.loo))["summary"]["held_out_mae_pct_of_fits_without_x_mean"]
    base = CorunModel.load()

    def alone_med(n):
        v = [g["ms"][0] / g.get("iters", 20) for g in groups if g["w"] == [n]]
        return float(np.median(v)) if v else None

    local = {n: alone_med(n) for n in base.names}
    variants = {}
    for tag in ("fitted_alone", "box_alone", "box_alone_no_fill"):
        m = base
        if tag.startswith("box_alone"):
            A = m.alone_ms.copy()
            for i, n in enumerate(m.names):
                if local.get(n):
                    A[i] = local[n]
            m = CorunModel(list(m.names), A, m.u.copy(), m.v.copy(), dict(m.meta))
        for x in extra:
            m = with_workload(m, x, alone_med(x), mfma_share(x), fill=None if tag.endswith("no_fill") else cu_fill(x))
        variants[tag] = m
    report = {"groups": os.path.relpath(os.path.abspath(a.groups), ROOT), "n_groups": len(groups),
              "held_out_mae_pct": held_out, "bar_pct": round(2 * held_out, 3), "per_workload": {},
              "fill_betas": fill_betas(base),
              "catalog_alone_box_over_fitted": {n: round(local[n] / float(base.alone_ms[base.index[n]]), 4)
                                                for n in base.names if local.get(n)}}
    for x in extra:
        test = [g for g in groups if x in g["w"] and len(g["w"]) >= 2]
        r = {"alone_ms_per_iter": round(alone_med(x), 5), "mfma_share": round(mfma_share(x), 4),
             "cu_fill": cu_fill(x),
             "test_groups": len(test), "neighbours": variants["fitted_alone"].meta["cold_start"][x]["neighbours"]}
        for tag, m in variants.items():
            xi = m.index[x]
            ext = [m.index[e] for e in extra]
            r[tag] = {"cold_start_x": errors(m, test, lambda w: w == xi),
                      "catalog_corunners": errors(m, test, lambda w: ~np.isin(w, ext) & (w >= 0))}
        report["per_workload"][x] = r
    xs = [r["box_alone"]["cold_start_x"]["mae_pct"] for r in report["per_workload"].values()]
    report["summary"] = {"cold_start_mae_pct": {x: r["box_alone"]["cold_start_x"]["mae_pct"]
                                                for x, r in report["per_workload"].items()},
                         "cold_start_mae_pct_without_fill": {x: r["box_alone_no_fill"]["cold_start_x"]["mae_pct"]
                                                             for x, r in report["per_workload"].items()},
                         "catalog_corunner_mae_pct": {x: r["box_alone"]["catalog_corunners"]["mae_pct"]
                                                      for x, r in report["per_workload"].items()},
                         "max_ratio_to_held_out": round(max(xs) / held_out, 3), "within_2x": bool(max(xs) <= 2 * held_out)}
    print(json.dumps(report["summary"], indent=1))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(report, open(a.out, "w"), indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
