"""Measure the MI355X configuration and interference matrices of the workload catalog.

The reference ships two matrices measured offline on A30/V100
(reference pkg/recommender/recommender/configurations_train.ods: throughput per
`<N>P_<GPU>` share; interference_train.ods: throughput lost per co-runner) and has no
code that produced them.  This tool produces the same two tables on
MI355X for `models.workloads.CATALOG`, with the native kernels and CU-masked streams:

  configurations_mi355x.tsv  rows = workloads, columns {1,2,4,8}P_MI355X:
      iterations/s of the workload alone on a 1/P CU share (hard CU mask of 8/P units)
  interference_mi355x.tsv    rows = workloads, columns = workloads:
      iterations/s the row workload loses on its quarter share while the column
      workload runs on another quarter (both hard-masked)

Output TSVs use the reference layout (first column `index`), so the recommender serves
them unchanged; missing cells (e.g. `--pairs` sampling) are imputed by its model.
Usage (GPU box): python -m k8s_gpu_scheduler_amd.models.profile --out k8s_gpu_scheduler_amd/data
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import random
import time
from typing import Dict, List, Optional

import numpy as np


def _time_pods(ex, runs) -> None:
    import torch
    ex.launch_epoch(runs)
    torch.cuda.synchronize()
    ex.collect(runs)


def profile(iters: int = 8, pairs: Optional[int] = None, seed: int = 0, names: Optional[List[str]] = None,
            repeats: int = 3):
    """Median of `repeats` timed runs per cell (alone and co-located alike, so interference
    = median alone - median co-located is not biased by the estimator)."""
    import torch
    from ..parallel.executor import DeviceExecutor, PodRun
    from . import workloads as W
    names = names or list(W.NAMES)
    ex = DeviceExecutor(0, use_cu_masks=True)
    shares = {1: (0, 8), 2: (0, 4), 4: (0, 2), 8: (0, 1)}
    # warm every stream / buffer
    ex.warm([PodRun(0, n, u0, k, 1) for n in names for (u0, k) in list(shares.values()) + [(2, 2)]])
    conf = np.zeros((len(names), 4))
    reps = max(1, repeats)
    for i, n in enumerate(names):
        for j, p in enumerate((1, 2, 4, 8)):
            u0, k = shares[p]
            samples = []
            for _ in range(reps):
                r = [PodRun(0, n, u0, k, iters)]
                _time_pods(ex, r)
                samples.append(r[0].throughput)
            conf[i, j] = float(np.median(samples))
    alone4 = conf[:, 2]
    intf = np.full((len(names), len(names)), np.nan)
    todo = list(itertools.product(range(len(names)), range(len(names))))
    if pairs:
        random.Random(seed).shuffle(todo)
        todo = todo[:pairs]
    for i, j in todo:
        samples = []
        for _ in range(reps):
            a = PodRun(0, names[i], 0, 2, iters)
            b = PodRun(1, names[j], 2, 2, iters * 4)      # co-runner outlives the victim
            _time_pods(ex, [b, a])
            samples.append(a.throughput)
        intf[i, j] = max(0.0, alone4[i] - float(np.median(samples)))
    ex.close()
    return names, conf, intf


def write_tables(out_dir: str, names: List[str], conf: np.ndarray, intf: np.ndarray, model: str = "MI355X") -> Dict[str, str]:
    from ..recommender.tables import Table
    os.makedirs(out_dir, exist_ok=True)
    c = Table(list(names), [f"{p}P_{model}" for p in (1, 2, 4, 8)], conf.astype(float))
    i = Table(list(names), list(names), intf.astype(float))
    cp = os.path.join(out_dir, "configurations_mi355x.tsv")
    ip = os.path.join(out_dir, "interference_mi355x.tsv")
    c.write_tsv(cp)
    i.write_tsv(ip)
    return {"configurations": cp, "interference": ip}


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(os.path.dirname(os.path.dirname(__file__)), "data"))
    ap.add_argument("--iters", type=int, default=16)
    ap.add_argument("--pairs", type=int, default=0, help="sample this many interference pairs (0 = all)")
    ap.add_argument("--repeats", type=int, default=3, help="timed runs per cell (median)")
    a = ap.parse_args(argv)
    t = time.time()
    names, conf, intf = profile(a.iters, a.pairs or None, repeats=a.repeats)
    paths = write_tables(a.out, names, conf, intf)
    print(json.dumps({"paths": paths, "seconds": round(time.time() - t, 1),
                      "conf_1P_min_max": [float(conf[:, 0].min()), float(conf[:, 0].max())]}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
