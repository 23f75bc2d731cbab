"""Leave-one-workload-out evaluation of the co-run model's cold start (models.coldstart).

For every catalog workload X: refit the co-run model on the MI355X groups WITHOUT X (every
group containing X removed), cold-start X from its alone profile only (median alone ms per
iteration of its 1-pod groups; its MFMA share; its CU fill unless --no-fill), and measure the throughput error on X's
measured co-run groups.  Compared with: the full fit's row for X (X seen in training) and the
roofline prior row.  Writes a JSON report (profiles/archive/r04_coldstart/).

    python tools/corun_coldstart_eval.py [--groups profiles/archive/r03_corun_v2/groups_2558_hostwait.json]
                                         [--jobs 6] [--out profiles/archive/r04_coldstart/loo.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def _err(model, groups, names, i):
    from k8s_gpu_scheduler_amd.models.corun import pack_groups
    wids, iters, mask, ms, st = pack_groups(groups, names, 4)
    t = model.batch_times(wids, iters, mask, st) - st
    sel = mask & (wids == i)
    tp, tm = iters / np.maximum(t, 1e-9) * 1e3, iters / np.maximum(ms, 1e-9) * 1e3
    return {"mae_pct": float(100 * np.abs(tp - tm)[sel].mean() / tm[sel].mean()),
            "mean_abs_log": float(np.abs(np.log(np.maximum(t, 1e-9) / np.maximum(ms, 1e-9)))[sel].mean()),
            "pods": int(sel.sum())}


def one(args):
    path, X, nfev, use_fill = args
    from k8s_gpu_scheduler_amd.models.coldstart import cu_fill, mfma_share, with_workload
    from k8s_gpu_scheduler_amd.models.corun import CorunModel, fit
    d = json.load(open(path))
    names = d["names"]
    groups = d["groups"]
    i = names.index(X)
    train = [g for g in groups if X not in g["w"]]
    test = [g for g in groups if X in g["w"] and len(g["w"]) >= 2]
    alone = [g["ms"][0] / g.get("iters", 20) for g in groups if g["w"] == [X]]
    m, rep = fit(train, names, max_nfev=nfev)
    cold = with_workload(m, X, float(np.median(alone)), mfma_share(X), fill=cu_fill(X) if use_fill else None)
    full = CorunModel.load()
    prior = CorunModel.prior(names)
    pr = CorunModel(names, m.alone_ms.copy(), m.u.copy(), m.v.copy())
    pr.alone_ms[i] = float(np.median(alone))
    pr.u[i], pr.v[i] = prior.u[i], prior.v[i]
    pr = CorunModel(names, pr.alone_ms, pr.u, pr.v)
    return X, {"cold_start": _err(cold, test, names, i), "fitted_with_x": _err(full, test, names, i),
               "prior_row": _err(pr, test, names, i), "fit_without_x_test": rep["test"],
               "neighbours": cold.meta["cold_start"][X]["neighbours"]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", default=os.path.join(ROOT, "profiles", "archive", "r03_corun_v2", "groups_2558_hostwait.json"))
    ap.add_argument("--jobs", type=int, default=6)
    ap.add_argument("--nfev", type=int, default=200)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "archive", "r04_coldstart", "loo.json"))
    ap.add_argument("--no-fill", action="store_true", help="cold start without the CU-fill scaling (round 4)")
    a = ap.parse_args()
    names = json.load(open(a.groups))["names"]
    with ProcessPoolExecutor(a.jobs) as ex:
        res = dict(ex.map(one, [(a.groups, X, a.nfev, not a.no_fill) for X in names]))
    cs = [r["cold_start"]["mae_pct"] for r in res.values()]
    fw = [r["fitted_with_x"]["mae_pct"] for r in res.values()]
    pr = [r["prior_row"]["mae_pct"] for r in res.values()]
    ho = [r["fit_without_x_test"]["mae_pct_of_mean"] for r in res.values()]
    summary = {"cold_start_mae_pct": {"mean": round(float(np.mean(cs)), 2), "median": round(float(np.median(cs)), 2),
                                      "max": round(float(np.max(cs)), 2)},
               "fitted_with_x_mae_pct_mean": round(float(np.mean(fw)), 2),
               "prior_row_mae_pct_mean": round(float(np.mean(pr)), 2),
               "held_out_mae_pct_of_fits_without_x_mean": round(float(np.mean(ho)), 2),
               "ratio_cold_to_held_out": round(float(np.mean(cs) / np.mean(ho)), 3)}
    print(json.dumps(summary, indent=1))
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"groups": os.path.relpath(a.groups, ROOT), "summary": summary, "per_workload": res}, f, indent=1)


if __name__ == "__main__":
    main()
