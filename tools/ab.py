"""Interleaved A/B driver for bench.py (replaces the per-study *_ab.sh scripts of rounds 1-2).

Every arm runs once per round, arms interleaved inside a round so box drift (clocks, other
tenants of the host) hits all arms alike; each run is its own bench.py process under a
time limit, and the driver stops at the first failure (no retries on a GPU box).

    python tools/ab.py --rounds 3 --steps 20 --warmup 5 \\
        --arm plain="--dist-single 0" --arm rccl="--dist-single 1" --out gpurun_out/ab_window

An arm is NAME=FLAGS; FLAGS may start with ENV=VALUE words, which go to that run's
environment (e.g. --arm q8="GPUSCHED_HW_QUEUES=8 --steps 60").  Writes per-run JSON and logs
under --out plus summary.json (median / min / max of value, ms_per_step, gpu_util_pct,
slo_attainment_pct, sol_pct.achievable per arm) and prints one line per run.
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys
from typing import Dict, List, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("value", "ms_per_step", "gpu_util_pct", "slo_attainment_pct", "sol_achievable")


def parse_arm(spec: str) -> Tuple[str, Dict[str, str], List[str]]:
    if "=" not in spec:
        raise SystemExit(f"--arm wants NAME=FLAGS, got {spec!r}")
    name, rest = spec.split("=", 1)
    env, flags = {}, []
    for w in shlex.split(rest):
        if not flags and "=" in w and not w.startswith("-"):
            k, v = w.split("=", 1)
            env[k] = v
        else:
            flags.append(w)
    return name, env, flags


def row(d: Dict) -> Dict[str, float]:
    return {"value": d.get("value"), "ms_per_step": d.get("ms_per_step"), "gpu_util_pct": d.get("gpu_util_pct"),
            "slo_attainment_pct": d.get("slo_attainment_pct"),
            "sol_achievable": (d.get("sol_pct") or {}).get("achievable")}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--arm", action="append", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--timeout", type=int, default=180, help="seconds per bench run")
    ap.add_argument("--out", default="gpurun_out/ab")
    a = ap.parse_args(argv)
    arms = [parse_arm(s) for s in a.arm]
    os.makedirs(a.out, exist_ok=True)
    results: Dict[str, List[Dict[str, float]]] = {n: [] for n, _, _ in arms}
    for r in range(a.rounds):
        for name, env, flags in arms:
            tag = f"{name}_r{r}"
            js, log = os.path.join(a.out, tag + ".json"), os.path.join(a.out, tag + ".log")
            cmd = ["timeout", "-k", "10", str(a.timeout), sys.executable, os.path.join(ROOT, "bench.py"),
                   "--steps", str(a.steps), "--warmup", str(a.warmup)] + flags + ["--out", js]
            with open(log, "w") as f:
                rc = subprocess.call(cmd, cwd=ROOT, env={**os.environ, **env}, stdout=f, stderr=subprocess.STDOUT)
            if rc != 0:
                print(f"{tag}: exit {rc} (see {log}); stopping", flush=True)
                return rc
            d = row(json.load(open(js)))
            results[name].append(d)
            print(tag, json.dumps(d), flush=True)
    summary = {}
    for name, rows in results.items():
        summary[name] = {}
        for k in FIELDS:
            v = [x[k] for x in rows if x.get(k) is not None]
            if v:
                summary[name][k] = {"median": round(statistics.median(v), 3), "min": min(v), "max": max(v)}
    json.dump({"rounds": a.rounds, "steps": a.steps, "warmup": a.warmup, "arms": {n: {"env": e, "flags": f}
               for n, e, f in arms}, "runs": results, "summary": summary}, open(os.path.join(a.out, "summary.json"),
                                                                              "w"), indent=1)
    print(json.dumps(summary), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
