"""Replay a co-run learner observation log (GPUSCHED_CORUN_LOG, written by a bench run) through
OnlineCorun refit variants and score each prequentially (every group predicted before it is
learned from), as the bench's interference_mae does.

    python tools/corun_replay.py LOG.json [variant ...]      variants: centred (default), uncentred, noscale
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from k8s_gpu_scheduler_amd.models import corun as C  # noqa: E402


def base_model():
    from k8s_gpu_scheduler_amd.parallel.podbench import ControlPlane
    cp = ControlPlane(1, 4, 20, 0, balance=1.0, plan_bursts=True, slo_objective="corun", learn_corun=True)
    return cp.corun.base


def replay(log, base, variant: str):
    os.environ["GPUSCHED_REFIT_VARIANT"] = variant
    on = C.OnlineCorun(base, refit_every=128, background=False)
    idx = {n: i for i, n in enumerate(log["names"])}
    remap = [base.wid(n) for n in log["names"]]
    for w, it, st, ms, tg in log["groups"]:
        on.observe_group([remap[x] for x in w], it, ms, st, tg)
    m = on.mae()
    return {k: (round(v, 2) if isinstance(v, float) else v) for k, v in m.items()}


def main() -> int:
    path = sys.argv[1]
    if path.endswith(".gz"):
        import gzip
        log = json.load(gzip.open(path, "rt"))
    else:
        log = json.load(open(path))
    variants = sys.argv[2:] or ["uncentred", "centred", "noscale"]
    base = base_model()
    for v in variants:
        print(v, json.dumps(replay(log, base, v)), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
