"""Co-run groups of workloads OUTSIDE the catalog, measured on MI355X, for the cold-start check
(models.coldstart).

Every catalog workload is built from the same two kernels (bf16 GEMM + HBM triad), so the
leave-one-workload-out check (tools/corun_coldstart_eval.py) cannot show transfer to a
different kernel mix.  models.workloads.EXTRA has two workloads with other mixes:

  fp8_llm_2048      three fp8 (OCP e4m3) GEMMs 2048 x 4096 x 4096 on the block-scaled MFMA
  triad_only_2048   three HBM stream passes of 2048 x 16384 floats, no GEMM at all

Groups are measured exactly as the co-run table was (models.corun.collect): the executor's
captured per-pod HIP graphs, Burstable pods on unmasked slot streams 0/2/4/6 with 2-unit GEMM
budgets, 20 iterations per pod, per-pod HIP-event wall time, the host waiting for each group.
Alone groups (1 pod) are the cold start's only input; the multi-pod groups (an extra workload
with 1-3 catalog co-runners, or both extras together) are what it is scored on.  Catalog
co-runners are timed too, so the same groups also give the fitted model's error on this box.

    python tools/corun_extra_groups.py [--groups-per 40] [--out gpurun_out/corun_extra_groups.json]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups-per", type=int, default=40)
    ap.add_argument("--alone-reps", type=int, default=6)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/corun_extra_groups.json")
    a = ap.parse_args(argv)
    q = int(os.environ.get("GPUSCHED_HW_QUEUES", "16"))
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < q <= 32:
        os.environ["GPU_MAX_HW_QUEUES"] = str(q)         # as models.corun collect / bench.py
    import torch
    from k8s_gpu_scheduler_amd import _native
    from k8s_gpu_scheduler_amd.models import workloads as W
    from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun
    _native.hip(required=True)
    extra = list(W.EXTRA)
    ex = DeviceExecutor(0, use_cu_masks=True)
    ex.use_graphs = True
    slots = (0, 2, 4, 6)
    ex.warm([PodRun(0, wl, u, 2, a.iters, masked=False) for wl in W.NAMES + extra for u in slots])

    def run(wls):
        runs = [PodRun(i, wl, slots[i], 2, a.iters, masked=False) for i, wl in enumerate(wls)]
        torch.cuda.synchronize()
        ref = torch.cuda.Event(enable_timing=True)
        ref.record()
        ex.launch_epoch(runs)
        ex.wait_all()
        torch.cuda.synchronize()
        ms = [r.start.elapsed_time(r.end) for r in runs]
        st = [ref.elapsed_time(r.start) for r in runs]
        s0 = min(st)
        return {"w": list(wls), "iters": a.iters, "ms": [round(x, 4) for x in ms],
                "start": [round(x - s0, 4) for x in st]}

    rng = random.Random(a.seed)
    weights = [1.0 / (1 + (i % 6)) for i in range(len(W.NAMES))]

    def draw() -> str:
        return rng.choices(W.NAMES, weights)[0] if rng.random() < 0.5 else rng.choice(W.NAMES)

    plan = []
    for _ in range(a.alone_reps):
        plan += [[x] for x in extra]
    for _ in range(3):
        plan += [[n] for n in W.NAMES]               # this box's catalog alone times
    for x in extra:
        for j in range(a.groups_per):
            k = 3 if j % 2 else rng.choice((1, 2))  # the bench's 4-pod shape half the time
            wls = [x] + [draw() for _ in range(k)]
            rng.shuffle(wls)
            plan.append(wls)
    for _ in range(a.groups_per // 4):
        wls = extra + [draw() for _ in range(rng.choice((0, 1, 2)))]
        rng.shuffle(wls)
        plan.append(wls)
    for wls in plan[:8]:                               # untimed warm-up
        run(wls)
    out, t0 = [], time.time()
    for i, wls in enumerate(plan):
        out.append(run(wls))
        if i % 40 == 0:
            print(f"[extra] {i}/{len(plan)} groups, {time.time() - t0:.1f}s", flush=True)
    ex.close()
    shares = {}
    from k8s_gpu_scheduler_amd.models.coldstart import mfma_share
    for x in extra:
        shares[x] = mfma_share(x)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump({"iters": a.iters, "names": list(W.NAMES) + extra, "extra": extra, "extra_mfma_share": shares,
               "groups": out}, open(a.out, "w"))
    print(json.dumps({"groups": len(out), "out": a.out}))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
