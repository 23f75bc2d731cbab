"""A long bench run (stability over thousands of epochs): runs bench.py as a child process and
reports the largest resident set of its processes next to the bench's JSON summary.

    python tools/long_bench.py --steps 3000 --out gpurun_out/longrun
"""
import argparse
import json
import os
import resource
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/longrun")
    ap.add_argument("--extra", default="", help="more bench.py flags (one string)")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    js = os.path.join(a.out, f"bench{a.steps}.json")
    trace = os.path.join(a.out, f"trace{a.steps}.json")
    env = dict(os.environ, GPUSCHED_BENCH_TRACE=trace)
    with open(os.path.join(a.out, f"bench{a.steps}.log"), "w") as log:
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", str(a.steps),
                            "--warmup", str(a.warmup), "--seed", str(a.seed), "--out", js, *a.extra.split()], stdout=log,
                           stderr=subprocess.STDOUT, env=env)
    rss_mb = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss / 1024
    if p.returncode != 0:
        print(json.dumps({"rc": p.returncode, "max_rss_mb": rss_mb}))
        return p.returncode
    d = json.load(open(js))
    out = {"steps": a.steps, "seed": a.seed, "value": d["value"], "ms_per_step": d["ms_per_step"],
           "slo_attainment_pct": d["slo_attainment_pct"], "sol_pct": d["sol_pct"],
           "timed_graph_captures_rank0": d.get("timed_graph_captures_rank0"),
           "effort_epochs": (d.get("planner") or {}).get("effort_epochs"), "max_rss_mb_child": round(rss_mb, 1),
           "extra": a.extra}
    for k in ("interference_mae", "corun_learner"):
        if k in d:
            out[k] = d[k]
    # pods completed per tenth of the run (GPU clock): does the rate drift over thousands of epochs?
    if os.path.exists(trace):
        ends = sorted(x[4] for x in json.load(open(trace))["pods"])
        n = len(ends)
        cuts = [ends[min(n - 1, (k * n) // 10)] for k in range(11)]
        out["pods_per_s_by_tenth"] = [round((n / 10) / max(cuts[k + 1] - cuts[k], 1e-9) * 1e3, 1) for k in range(10)]
        os.remove(trace)
    print(json.dumps(out))
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
