"""How much of a co-run epoch is GEMM/HBM overlap?  Runs the bench's pod mix (4 Burstable
pods of 2 CU units, random catalog workloads, 20 iterations) through the real
DeviceExecutor with each pod's op list restricted to (a) everything, (b) GEMMs only,
(c) triads only, and (d) everything on ONE stream (no co-run).  If full ~= gemm + triad the
pods do not overlap compute with HBM streaming; the floor is max(gemm, triad).
Writes gpurun_out/overlap.json."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402


def run(ex, epochs, keep):
    saved = {}
    for k, b in ex._bufs.items():
        saved[k] = b.ops
        b.ops = [(o, t) for o, t in b.ops if keep(o)]
    try:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for ep in epochs:
            ex.launch_epoch(ep)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / len(epochs) * 1e3
    finally:
        for k, b in ex._bufs.items():
            b.ops = saved[k]


def main():
    ex = DeviceExecutor(0)
    ex.use_graphs = False
    rng = random.Random(1)
    weights = [1.0 / (1 + (i % 6)) for i in range(len(W.NAMES))]
    epochs = [[PodRun(4 * e + i, rng.choices(W.NAMES, weights)[0], 2 * i, 2, 20, masked=False) for i in range(4)]
              for e in range(12)]
    serial = [[PodRun(r.pod_id, r.workload, 0, 8, r.iters, masked=False) for r in ep] for ep in epochs]
    ex.warm([PodRun(0, wl, u, 2, 1, masked=False) for wl in W.NAMES for u in (0, 2, 4, 6)])
    ex.warm([PodRun(0, wl, 0, 8, 1, masked=False) for wl in W.NAMES])
    cases = {
        "full": (epochs, lambda o: True),
        "gemm_only": (epochs, lambda o: o.kind == "gemm"),
        "triad_only": (epochs, lambda o: o.kind != "gemm"),
        "full_one_stream": (serial, lambda o: True),
        "gemm_one_stream": (serial, lambda o: o.kind == "gemm"),
        "triad_one_stream": (serial, lambda o: o.kind != "gemm"),
    }
    res = {k: [] for k in cases}
    for rnd in range(4):
        for k, (eps, keep) in cases.items():
            ms = run(ex, eps, keep)
            if rnd:
                res[k].append(round(ms, 3))
        print(rnd, {k: v[-1] for k, v in res.items() if v}, flush=True)
    gf = sum(W.CATALOG[r.workload].flops for ep in epochs for r in ep) * 20 / len(epochs)
    tb = sum(o.bytes for ep in epochs for r in ep for o in W.CATALOG[r.workload].ops if o.kind != "gemm") * 20 / len(epochs)
    out = {k: {"ms_per_epoch": v, "best": min(v)} for k, v in res.items()}
    out["per_epoch_work"] = {"tflop": gf / 1e12, "triad_gb": tb / 1e9}
    b = {k: out[k]["best"] for k in cases}
    out["derived"] = {"triad_tbps_corun": tb / 1e9 / b["triad_only"], "gemm_tflops_corun": gf / 1e9 / b["gemm_only"],
                      "overlap_gain_ms": b["gemm_only"] + b["triad_only"] - b["full"]}
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/overlap.json", "w"), indent=1)
    print(json.dumps(out, indent=1))
    # phase staggering: slot k starts its op cycle at op k (same ops, rotated order)
    def rotated(keep_all):
        saved = {k: b.ops for k, b in ex._bufs.items()}
        for (wl, u0, n), b in ex._bufs.items():
            r = (u0 // 2) % max(len(b.ops), 1)
            b.ops = b.ops[r:] + b.ops[:r]
        try:
            return run(ex, epochs, keep_all)
        finally:
            for k, b in ex._bufs.items():
                b.ops = saved[k]
    rot = []
    for rnd in range(4):
        f = run(ex, epochs, lambda o: True)
        g = rotated(lambda o: True)
        if rnd:
            rot.append((round(f, 3), round(g, 3)))
    out["rotation_full_vs_rotated_ms"] = rot
    print("rotation", rot, flush=True)
    from k8s_gpu_scheduler_amd import _native
    hip = _native.hip(required=True)
    json.dump(out, open("gpurun_out/overlap.json", "w"), indent=1)
    if os.environ.get("OVERLAP_SHORT"):
        ex.close()
        return
    # stream-kernel launch shape sweep under co-run: (triad variant, blocks)
    sweep = {}
    configs = [(6, 0), (3, 256), (3, 1024), (4, 256)]
    for rnd in range(3):
        for v, nb in configs:
            hip.set_triad_variant(v)
            ex.triad_blocks = nb
            f = run(ex, epochs, lambda o: True)
            t = run(ex, epochs, lambda o: o.kind != "gemm")
            if rnd:
                sweep.setdefault(f"v{v}_b{nb}", []).append((round(f, 3), round(t, 3)))
    hip.set_triad_variant(6)
    ex.triad_blocks = 0
    out["triad_sweep_full_vs_triad_only_ms"] = {k: [min(x[0] for x in v), min(x[1] for x in v)] for k, v in sweep.items()}
    # GEMM tile (forced) under co-run with the HBM phases: 0 = the share-based picker
    tiles = {}
    for rnd in range(3):
        for t in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9):
            hip.set_gemm_tile(t)
            f = run(ex, epochs, lambda o: True)
            if rnd:
                tiles.setdefault(f"tile{t}", []).append(round(f, 3))
    hip.set_gemm_tile(0)
    out["gemm_tile_full_ms"] = {k: min(v) for k, v in tiles.items()}
    print(sorted(out["gemm_tile_full_ms"].items(), key=lambda kv: kv[1]), flush=True)
    json.dump(out, open("gpurun_out/overlap.json", "w"), indent=1)
    for k, v in sorted(out["triad_sweep_full_vs_triad_only_ms"].items(), key=lambda kv: kv[1][0]):
        print(k, v, flush=True)
    ex.close()


if __name__ == "__main__":
    main()
