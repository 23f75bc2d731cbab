"""Pipelined virtual node: an 8-GPU node's placement streams replayed through the bench's real
launch-ahead slot pipeline on ONE MI355X, SLOs counted from what actually co-ran.

tools/virtual_node_bench.py runs each virtual GPU's epoch group in isolation (launch, wait,
next group): pods start together and never overlap the previous epoch's tail, which is where
the co-run planner's model is exact.  The driver's N-GPU bench is different: every rank
keeps `--lookahead` epochs in flight, each CU slot's stream runs its pods back to back, and a
pod's co-runners are partly the neighbouring epochs' pods.  This tool measures placement
policies in THAT setting:

  1. schedule (CPU, a child process): the bench's control plane for an N-GPU node
     (`bench.py --sim --sim-model --gpus N`), whose feedback -- per-pod intervals for the
     planner's slot timelines, busy time for its backlog, co-run observations -- comes from
     the co-run model's pipeline simulation (parallel.modelpipe); every epoch's placements
     (GPU, CU slot, workload, SLO) are dumped (--dump-placements);
  2. replay (the MI355X): for every virtual GPU in turn, its placement stream runs through
     the bench's own executor (parallel.podbench.gpu_executor: slot streams, HIP graphs,
     the native MFMA / HBM kernels) with the bench's launch-ahead pipeline, so each pod
     co-runs with exactly the pods its GPU's pipeline puts next to it; pod throughput and SLO
     come from its HIP events.  Policies alternate per virtual GPU (same arrivals: same seed).

Reported per policy: the hardware SLO attainment and pods/s (the node's pods over its slowest
virtual GPU's busy span), next to the simulation's own numbers.  The replay is open loop
(placements were decided on simulated feedback); `--replay sim` runs step 2 on the model
pipeline instead (CPU check of the tool itself).

    python tools/pipelined_vn.py [--gpus 8] [--epochs 48] [--seeds 0 1 2] [--out gpurun_out/pvn.json]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
_q = int(os.environ.get("GPUSCHED_HW_QUEUES", "16"))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _q <= 32:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_q)

import numpy as np  # noqa: E402

POLICIES = {
    # the reference's behaviour in this framework: Score (co-run SLO constraint + balance), no plan
    "greedy": ["--plan-bursts", "0"],
    # the bench default: burst planner on the co-run model, backlog carry, slot planning
    "planner": [],
    # the cheaper planning levels the adaptive control plane falls back to at 8 GPUs
    # (planner.BurstPlanner.EFFORT_LEVELS: 1 = a quarter of the sweeps, phantoms kept; 2 = half the
    # sweeps, no phantoms, lpt slots, no pipeline evaluation; 3 = also one sweep per phase)
    "planner-e1": ["--plan-effort", "1"],
    "planner-e2": ["--plan-effort", "2"],
    "planner-e3": ["--plan-effort", "3"],
    # how far a GPU's predicted time may exceed the balanced plan's slowest GPU to meet more SLOs
    "planner-tol05": ["--plan-tolerance", "0.5"],
    "planner-tol08": ["--plan-tolerance", "0.8"],
    # the model error the planner's expected-SLO objective assumes (default 0.05, the held-out
    # error of isolated groups; pipelined predictions are looser)
    "planner-sig10": ["--corun-sigma", "0.1"],
    "planner-sig20": ["--corun-sigma", "0.2"],
    "random": ["--policy", "random"],
    # alternative effort-level tables (planner.BurstPlanner.EFFORT_LEVELS) at level 1: phantoms
    # kept with 2 sweeps (a) or 1 sweep (c); "-e1old": round 5's first level 1 (no phantoms, 2 sweeps)
    "planner-e1a": ["--plan-effort", "1"],
    "planner-e1c": ["--plan-effort", "1"],
    "planner-e1old": ["--plan-effort", "1"],
}
POLICY_ENV = {
    "planner-e1a": {"GPUSCHED_EFFORT_LEVELS": "1,1,1,1;2,1,1,1;2,0,0,0;0,0,0,0"},
    "planner-e1c": {"GPUSCHED_EFFORT_LEVELS": "1,1,1,1;4,1,1,1;2,0,0,0;0,0,0,0"},
    "planner-e1old": {"GPUSCHED_EFFORT_LEVELS": "1,1,1,1;2,0,1,1;2,0,0,0;0,0,0,0"},
}


def schedule(policy: str, flags, gpus: int, epochs: int, warmup: int, seed: int, path: str) -> dict:
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--sim", "--sim-model", "--gpus", str(gpus),
           "--steps", str(epochs), "--warmup", str(warmup), "--seed", str(seed), "--dump-placements", path, *flags]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=dict(os.environ, **POLICY_ENV.get(policy, {})))
    if p.returncode != 0:
        raise RuntimeError(f"scheduling {policy} failed: {p.stderr[-2000:]}")
    with open(path) as f:
        return json.load(f)


def replay_gpu(ex, epochs, g: int, lookahead: int, release=None, clock=time.perf_counter) -> dict:
    """One virtual GPU's placement stream through the launch-ahead pipeline on `ex`.

    release[e] (ms after the replay's start, optional): the earliest host time epoch e may be
    launched -- the coupled node's placement broadcast, which waits until EVERY GPU collected
    epoch e - lookahead - 1.  Returns the SLO counts of the timed epochs and, per epoch, the
    host time its pods were collected (`done_ms`)."""
    from k8s_gpu_scheduler_amd.parallel.podbench import _runs_for
    pending = collections.deque()
    timed_runs = []
    done = [0.0] * len(epochs)
    sim = hasattr(ex, "elapsed_ms")        # the model pipeline: its simulated host clock (ms)
    if sim:
        def clock():
            return ex.now / 1e3
    t0 = clock()

    def collect():
        e, runs = pending.popleft()
        ex.wait_epoch(runs)
        done[e] = (clock() - t0) * 1e3

    for e, ep in enumerate(epochs):
        arr = np.asarray(ep["arr"], dtype=np.int32)
        runs = _runs_for(arr, g)
        for r in runs:
            r.gpu = 0                                # every virtual GPU replays on device 0
        if release is not None:
            if sim:
                ex.now = max(ex.now, t0 * 1e3 + release[e])
            while (clock() - t0) * 1e3 < release[e]:
                pass                                 # host-side gate (sub-10 us on a spinning core)
        ex.launch_epoch(runs)
        pending.append((e, runs))
        if ep["timed"]:
            timed_runs += runs
        while len(pending) > lookahead:
            collect()
    while pending:
        collect()
    ex.wait_all()
    ok = 0
    starts, ends = [], []
    per_wl = collections.defaultdict(lambda: [0, 0])
    for r in timed_runs:
        r.ms = r.start.elapsed_time(r.end)
        met = r.slo <= 0 or r.throughput >= r.slo
        ok += met
        per_wl[r.workload][0] += met
        per_wl[r.workload][1] += 1
        starts.append(ex.clock.elapsed_time(r.start))
        ends.append(ex.clock.elapsed_time(r.end))
    span = (max(ends) - min(starts)) if timed_runs else 0.0
    return {"pods": len(timed_runs), "slo_ok": ok, "span_ms": span, "per_workload": dict(per_wl), "done_ms": done}


def coupled_release(done_per_gpu, lookahead: int):
    """release[e] = the latest GPU's collect time of epoch e - lookahead - 1 (0 before)."""
    n = len(done_per_gpu[0])
    return [max(d[e - lookahead - 1] for d in done_per_gpu) if e - lookahead - 1 >= 0 else 0.0 for e in range(n)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seeds", type=int, nargs="+", default=[0])
    ap.add_argument("--policies", nargs="+", default=["greedy", "planner", "random"], choices=list(POLICIES))
    ap.add_argument("--replay", default="gpu", choices=["gpu", "sim"])
    ap.add_argument("--passes", type=int, default=3,
                    help="replay passes: 1 = free-running virtual GPUs; more = launches gated by the coupled "
                         "node's broadcast times from the previous pass")
    ap.add_argument("--out", default="gpurun_out/pipelined_vn.json")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="pvn")
    plans = {}
    t0 = time.time()
    # 1. every schedule first, in child processes (before this process touches the GPU)
    for seed in a.seeds:
        for pol in a.policies:
            plans[(seed, pol)] = schedule(pol, POLICIES[pol], a.gpus, a.epochs, a.warmup, seed,
                                          os.path.join(tmp, f"{pol}_s{seed}.json"))
            print(f"scheduled {pol} seed {seed}: sim {plans[(seed, pol)]['sim']} ({time.time() - t0:.0f} s)",
                  flush=True)
    # 2. replay
    from k8s_gpu_scheduler_amd.models import workloads as W
    if a.replay == "gpu":
        import torch
        from k8s_gpu_scheduler_amd.parallel.executor import PodRun
        from k8s_gpu_scheduler_amd.parallel.podbench import build_parser, gpu_executor
        assert torch.cuda.is_available(), "--replay gpu needs a GPU"
        ex = gpu_executor(build_parser().parse_args([]), 0)
        ex.warm([PodRun(0, wl, u, 2, 20, masked=False) for wl in W.NAMES for u in (0, 2, 4, 6)])

        def executor():
            return ex
    else:
        from k8s_gpu_scheduler_amd.parallel.modelpipe import ModelPipelineExecutor

        def executor():
            return ModelPipelineExecutor(noise=0.05, seed=int(time.time()) % 1000)
    res = {}
    for seed in a.seeds:
        acc = {pol: None for pol in a.policies}
        rel = {pol: None for pol in a.policies}
        # pass 0: every virtual GPU free-running; pass k: launches gated by the coupled node's
        # broadcast times computed from pass k-1's collect times (a fixed-point iteration)
        for ps in range(a.passes):
            cur = {pol: [] for pol in a.policies}
            for g in range(a.gpus):
                for pol in a.policies:          # alternate policies per virtual GPU
                    d = plans[(seed, pol)]
                    cur[pol].append(replay_gpu(executor(), d["epochs"], g, d["lookahead"], rel[pol]))
            for pol in a.policies:
                rel[pol] = coupled_release([x["done_ms"] for x in cur[pol]], plans[(seed, pol)]["lookahead"])
                acc[pol] = cur[pol]
            print(f"seed {seed} pass {ps}:", {pol: round(100.0 * sum(x["slo_ok"] for x in cur[pol]) /
                                                       max(sum(x["pods"] for x in cur[pol]), 1), 2)
                                              for pol in a.policies}, flush=True)
        for pol in a.policies:
            per = acc[pol]
            pods = sum(x["pods"] for x in per)
            ok = sum(x["slo_ok"] for x in per)
            slow = max(x["span_ms"] for x in per)
            t_end = max(x["done_ms"][-1] for x in per)
            wl = collections.defaultdict(lambda: [0, 0])
            for x in per:
                for k, (m, n) in x["per_workload"].items():
                    wl[k][0] += m
                    wl[k][1] += n
            res.setdefault(pol, []).append({
                "seed": seed, "hw_slo_attainment_pct": round(100.0 * ok / max(pods, 1), 2),
                "hw_pods_per_s": round(pods / max(slow, 1e-9) * 1e3, 1),
                "hw_pods_per_s_mean_gpu": round(pods / max(np.mean([x["span_ms"] for x in per]), 1e-9) * 1e3, 1),
                "coupled_end_ms": round(t_end, 2),
                "span_ms_per_gpu": [round(x["span_ms"], 2) for x in per], "pods": pods,
                "sim_pods_per_s": plans[(seed, pol)]["sim"]["value"],
                "sim_slo_attainment_pct": plans[(seed, pol)]["sim"]["slo_attainment_pct"],
                "slo_by_workload": {k: [m, n] for k, (m, n) in sorted(wl.items())}})
        print(json.dumps({pol: {k: v for k, v in res[pol][-1].items() if k not in ("slo_by_workload", "span_ms_per_gpu")}
                          for pol in a.policies}), flush=True)
    summary = {}
    base = res.get("greedy")
    for pol, rows in res.items():
        s = {"hw_slo_attainment_pct": round(float(np.mean([r["hw_slo_attainment_pct"] for r in rows])), 2),
             "hw_pods_per_s": round(float(np.mean([r["hw_pods_per_s"] for r in rows])), 1),
             "sim_slo_attainment_pct": round(float(np.mean([r["sim_slo_attainment_pct"] for r in rows])), 2),
             "sim_pods_per_s": round(float(np.mean([r["sim_pods_per_s"] for r in rows])), 1)}
        if base:
            s["hw_pods_per_s_vs_greedy"] = round(s["hw_pods_per_s"] / max(np.mean([r["hw_pods_per_s"] for r in base]),
                                                                       1e-9), 4)
        summary[pol] = s
    print(json.dumps(summary), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"gpus": a.gpus, "epochs": a.epochs, "warmup": a.warmup, "seeds": a.seeds, "replay": a.replay,
                   "note": "schedules made on the co-run model's pipeline simulation (open loop), each virtual "
                           "GPU's placement stream replayed through the bench's launch-ahead slot pipeline",
                   "summary": summary, "runs": res}, f, indent=1)


if __name__ == "__main__":
    main()
