"""Placement quality of an 8-GPU node, measured on ONE MI355X ("virtual node").

The driver's 8-GPU bench couples the ranks through the per-epoch placement broadcast, so an
epoch takes as long as its slowest GPU.  How long a GPU takes depends on WHICH four pods
the scheduler put on it (their work and how well their GEMM / HBM phases overlap).  This
tool runs the bench's control plane for an 8-GPU node (apiserver + scheduler + Poisson
arrivals, `parallel.podbench.ControlPlane`) and executes each of the 8 GPUs' pod groups
of every epoch on the one real GPU in turn (co-running, as on its own GPU), timing each
group with HIP events.  Per epoch it reports the slowest group (the coupled 8-GPU epoch
time), the mean group (the work-conserving bound), the node's epoch time when the measured
group times are replayed through the bench's 2-deep launch-ahead pipeline (ranks meet only
at the placement broadcast, so per-epoch imbalance averages out) and the SLO attainment, for placement policies side by side (interleaved per epoch, same arrivals):

  * greedy (balance + LPT, the reference's pairwise interference terms)
  * corun (Score under the multi-way co-run model's SLO constraint, models.corun)
  * corun_plan_tXX (burst planner on the co-run model: balanced group makespans, then the
    most predicted SLOs met within XX % of the balanced plan's slowest GPU)
  * planned (`planBursts` on the pairwise table; `planned_t0` with no load tolerance,
    `planned_load` with the load-first objective)
  * random

    python tools/virtual_node_bench.py [--epochs 12] [--out gpurun_out/virtual_node.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
# one HW queue per pod stream, as bench.py (before HIP initialises)
_q = int(os.environ.get("GPUSCHED_HW_QUEUES", "16"))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _q <= 32:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_q)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.podbench import (COST0, POD0, SMI0, TELE, ControlPlane, _cost_rows,  # noqa: E402
                                                     _pod_rows, _runs_for)

N_GPUS = 8
POLICIES = {
    "greedy": dict(balance=1.0, plan_bursts=False),
    "planned": dict(balance=1.0, plan_bursts=True, plan_tolerance=0.05),
    "planned_t0": dict(balance=1.0, plan_bursts=True, plan_tolerance=0.0),
    "planned_load": dict(balance=1.0, plan_bursts=True, plan_objective="load"),
    "random": dict(policy="random", balance=0.0, plan_bursts=False),
    "corun": dict(balance=1.0, plan_bursts=False, slo_objective="corun"),
    # corun_plan_tTT[_sSS]: burst planner on the co-run model, load tolerance TT %, soft
    # objective with model-error sigma 0.SS (none = hard SLO counts)
    **{f"corun_plan_t{t:02d}" + (f"_s{sg:02d}" if sg else ""):
       dict(balance=1.0, plan_bursts=True, plan_tolerance=t / 100.0, slo_objective="corun", corun_sigma=sg / 100.0)
       for t in (5, 10, 20, 30, 40, 50) for sg in (0, 3, 5, 8, 10)},
    # ..._cCC: backlog carried between bursts, decay 0.CC per burst (c100 = no decay)
    **{f"corun_plan_t{t:02d}_s05_c{c:03d}":
       dict(balance=1.0, plan_bursts=True, plan_tolerance=t / 100.0, slo_objective="corun", corun_sigma=0.05,
            plan_carry=c / 100.0)
       for t in (20, 30, 40, 50) for c in (90, 95, 100)},
    # the same without the measured busy-time feedback into the backlog
    **{f"corun_plan_t{t:02d}_s05_c100_nofb":
       dict(balance=1.0, plan_bursts=True, plan_tolerance=t / 100.0, slo_objective="corun", corun_sigma=0.05,
            plan_carry=1.0, plan_feedback=False)
       for t in (20, 30, 40)},
    # roofline complementarity term (GPU plugin weightComplement) on top of greedy
    "greedy_comp": dict(balance=1.0, plan_bursts=False, complement=1.0),
    "greedy_comp3": dict(balance=1.0, plan_bursts=False, complement=3.0),
}


from k8s_gpu_scheduler_amd.models.corun import CorunModel  # noqa: E402

MODEL = CorunModel.load()      # the shipped co-run model: predictions logged next to measurements


def run_group(ex: DeviceExecutor, runs):
    """Run one virtual GPU's pods co-located on the real GPU; returns wall ms."""
    if not runs:
        return 0.0
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    s.record()
    ex.launch_epoch(runs)
    ex.wait_all()         # host-side: a stream-wait here would slow one pod stream (executor.wait_all)
    for r in runs:
        r.ms = r.start.elapsed_time(r.end)
    return max(s.elapsed_time(r.end) for r in runs)


GROUPS: list = []      # per group: policy, workloads, wall ms, per pod (SLO, achieved, predicted), for --dump-groups


SIM = {"on": False, "sigma": 0.05, "rng": None, "speed": []}


def sim_group(runs, g: int = 0) -> float:
    """--simulate: the co-run model stands in for the GPU (each pod's predicted wall time
    times a lognormal error of sigma, its size on held-out groups); CPU-only policy studies."""
    if not runs:
        return 0.0
    t = MODEL.group_times([MODEL.wid(r.workload) for r in runs], [r.iters for r in runs])
    t = t * np.exp(SIM["rng"].normal(0.0, SIM["sigma"], len(runs)))
    if g < len(SIM["speed"]):
        t = t * SIM["speed"][g]             # a GPU slower (> 1) or faster than the model's
    for r, x in zip(runs, t):
        r.ms = float(x)
    return float(t.max())


def epoch(cp: ControlPlane, ex: DeviceExecutor, arr: np.ndarray, tag: str = ""):
    walls, per_gpu = [], np.zeros((N_GPUS, TELE))
    per_gpu[:, SMI0:] = -1.0          # one real GPU stands in for eight: no per-GPU amd-smi view
    ok = n = 0
    for g in range(N_GPUS):
        runs = _runs_for(arr, g)
        walls.append(sim_group(runs, g) if SIM["on"] else run_group(ex, runs))
        pred = [None] * len(runs)
        model = MODEL
        if model is not None and runs:
            pred = [round(float(x), 1) for x in model.group_tput([model.wid(r.workload) for r in runs],
                                                                 [r.iters for r in runs])]
        GROUPS.append({"policy": tag, "epoch": cp.epoch, "w": [r.workload for r in runs], "wall_ms": round(walls[-1], 4),
                       "slo": [round(r.slo, 1) for r in runs], "tput": [round(r.throughput, 1) for r in runs],
                       "pred": pred})
        for r in runs:
            per_gpu[g, :4] += (r.ms * r.n_units, 1, 1 if r.throughput >= r.slo else 0,
                               W.CATALOG[r.workload].hbm_gib)
            ok += r.slo <= 0 or r.throughput >= r.slo
            n += 1
        per_gpu[g, COST0:POD0] = _cost_rows(runs).ravel()
        per_gpu[g, POD0:SMI0] = _pod_rows(runs)
    cp.update_telemetry(per_gpu, max(walls))
    return walls, ok, n


def pipelined_ms(t: np.ndarray, lookahead: int) -> float:
    """Replay measured group times t[epoch][gpu] through the bench's launch-ahead pipeline:
    epoch e's placement broadcast waits until every rank collected epoch e-L-1, a GPU starts
    an epoch when it has finished its previous one and has the placement.  Returns ms per
    epoch of the whole node."""
    fin = np.zeros(t.shape[1])
    hist, bc = [], 0.0
    for e in range(len(t)):
        if e - lookahead - 1 >= 0:
            bc = max(bc, float(hist[e - lookahead - 1].max()))
        fin = np.maximum(fin, bc) + t[e]
        hist.append(fin.copy())
    return float(fin.max()) / max(len(t), 1)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8, help="GPUs of the virtual node")
    ap.add_argument("--epochs", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/virtual_node.json")
    ap.add_argument("--dump-groups", default="", help="write every group's workloads and wall ms (JSON)")
    ap.add_argument("--policies", nargs="+", default=["greedy", "corun", "corun_plan_t10", "random"],
                    choices=sorted(POLICIES))
    ap.add_argument("--simulate", action="store_true",
                    help="no GPU: group times from the co-run model with lognormal error (--sim-sigma)")
    ap.add_argument("--sim-sigma", type=float, default=0.05)
    ap.add_argument("--sim-speed", default="", help="per-GPU time multipliers, comma-separated (e.g. 1.06,1,1)")
    a = ap.parse_args()
    SIM.update(on=a.simulate, sigma=a.sim_sigma, rng=np.random.default_rng(a.seed),
               speed=[float(x) for x in a.sim_speed.split(",") if x])
    global N_GPUS
    N_GPUS = a.gpus
    policies = {k: POLICIES[k] for k in a.policies}
    cps = {k: ControlPlane(n_gpus=N_GPUS, pods_per_gpu=4, iters=20, seed=a.seed, **kw) for k, kw in policies.items()}
    ex = None
    if not a.simulate:
        ex = DeviceExecutor(0, use_cu_masks=True)
        ex.use_graphs = True            # as the bench (and the co-run model's measurements)
        ex.warm([PodRun(0, wl, u, 2, 20, masked=False) for wl in W.NAMES for u in (0, 2, 4, 6)])
    stats = {k: {"max_ms": [], "mean_ms": [], "walls": [], "ok": 0, "n": 0} for k in policies}
    for e in range(a.warmup + a.epochs):
        for k, cp in cps.items():
            cp.finish_live()
            arr = cp.schedule_epoch()
            walls, ok, n = epoch(cp, ex, arr, k)
            if e >= a.warmup:
                st = stats[k]
                st["max_ms"].append(max(walls))
                st["mean_ms"].append(statistics.mean(walls))
                st["walls"].append(walls)
                st["ok"] += ok
                st["n"] += n
        print(f"epoch {e}", {k: round(v["max_ms"][-1], 2) for k, v in stats.items() if v["max_ms"]}, flush=True)
    out = {}
    for k, st in stats.items():
        mx, mn = statistics.mean(st["max_ms"]), statistics.mean(st["mean_ms"])
        out[k] = {"epoch_ms_slowest_gpu": round(mx, 3), "epoch_ms_mean_gpu": round(mn, 3),
                  "imbalance": round(mx / mn, 4), "pods_per_s_coupled": round(4 * N_GPUS / mx * 1e3, 1),
                  "slo_attainment_pct": round(100.0 * st["ok"] / max(st["n"], 1), 2), "pods": st["n"],
                  "interference_mae": cps[k].interference_mae(),
                  "epoch_ms_pipelined_l2": round(pipelined_ms(np.array(st["walls"]), 2), 3),
                  # what paces the bench: its 2-deep launch-ahead pipeline over these group times
                  "pods_per_s_pipelined_l2": round(4 * N_GPUS / pipelined_ms(np.array(st["walls"]), 2) * 1e3, 1),
                  "epoch_ms_pipelined_l3": round(pipelined_ms(np.array(st["walls"]), 3), 3),
                  "epoch_ms_pipelined_l4": round(pipelined_ms(np.array(st["walls"]), 4), 3),
                  "walls_ms": [[round(x, 3) for x in w] for w in st["walls"]]}
    print(json.dumps(out), flush=True)
    if a.dump_groups:
        json.dump(GROUPS, open(a.dump_groups, "w"))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump({"note": "each virtual GPU's 4 pods co-run on the one real MI355X in turn; coupled N-GPU epoch = "
                       "slowest group; policies interleaved per epoch, same seed", "gpus": N_GPUS, "epochs": a.epochs,
               "simulated": ({"model": getattr(MODEL, "version", ""), "sigma": a.sim_sigma, "speed": SIM["speed"]}
                             if a.simulate else False),
               "results": out}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
