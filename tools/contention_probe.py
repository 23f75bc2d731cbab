"""GEMM x HBM-stream contention probe (one MI355X).

Why do co-running GEMM and stream-triad pods barely overlap (profiles/archive/r01_overlap_study.json:
full 8.10 ms vs GEMM-only 2.86 + triad-only 5.74)?  Two candidate causes:
  (1) CU contention -- the kernels compete for wave slots / VGPRs / LDS on the same CUs;
  (2) memory-system contention -- the saturated HBM stream inflates the GEMM's load latency
      even when the two run on disjoint CUs.
Each case runs a GEMM loop on one stream and a triad loop on another, alone and together,
with and without disjoint CU masks, and reports each side's rate.  Also sweeps the triad
launch shape and the GEMM tile under full sharing.  Writes gpurun_out/contention.json.
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402
from k8s_gpu_scheduler_amd.ops.cumask import MaskedStream  # noqa: E402
from k8s_gpu_scheduler_amd.plugins.gpu.devices import cu_slice_mask  # noqa: E402

hip = _native.hip(required=True)
dev = torch.device("cuda", 0)
M = N = K = int(os.environ.get("PROBE_GEMM", "2048"))
NF = int(os.environ.get("PROBE_TRIAD_FLOATS", str(4096 * 16384)))
a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
bt = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
c = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
bias = torch.zeros(N, device=dev)
x, y, z = (torch.ones(NF, device=dev) for _ in range(3))
GF = 2.0 * M * N * K
TB = 12.0 * NF


def plain():
    return torch.cuda.Stream(device=dev)


class S:
    def __init__(self, units=None, priority=0):
        if units is None:
            self.ms, self.stream = None, torch.cuda.Stream(device=dev, priority=priority)
        else:
            self.ms = MaskedStream(cu_slice_mask(units[0], units[1] - units[0]), 0)
            self.stream = self.ms.stream


def enqueue_gemm(st, n, budget=0):
    for _ in range(n):
        loadgen.gemm(a, bt, out=c, bias=bias, relu=True, stream=st, cu_budget=budget)


def enqueue_triad(st, n, blocks=0):
    for _ in range(n):
        loadgen.triad(x, y, z, 1.0001, blocks=blocks, stream=st)


def timed(jobs):
    """jobs: list of (stream, enqueue fn).  Returns per-job ms from a common start."""
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    ends = []
    side = torch.cuda.Stream(device=dev)
    start.record(side)
    for st, fn in jobs:
        st.wait_event(start)
        fn(st)
        e = torch.cuda.Event(enable_timing=True)
        e.record(st)
        ends.append(e)
    torch.cuda.synchronize()
    return [start.elapsed_time(e) for e in ends]


def case(name, gs, ts, ng, nt, gbudget=0, tblocks=0, reps=3):
    best = None
    for _ in range(reps):
        g_alone = timed([(gs.stream, lambda s: enqueue_gemm(s, ng, gbudget))])[0]
        t_alone = timed([(ts.stream, lambda s: enqueue_triad(s, nt, tblocks))])[0]
        g_co, t_co = timed([(gs.stream, lambda s: enqueue_gemm(s, ng, gbudget)),
                            (ts.stream, lambda s: enqueue_triad(s, nt, tblocks))])
        r = (g_alone, t_alone, g_co, t_co)
        if best is None or max(g_co, t_co) < max(best[2], best[3]):
            best = r
    g_alone, t_alone, g_co, t_co = best
    out = {"gemm_alone_tf": round(GF * ng / g_alone / 1e9, 1), "triad_alone_tbps": round(TB * nt / t_alone / 1e9, 2),
           "gemm_co_tf": round(GF * ng / g_co / 1e9, 1), "triad_co_tbps": round(TB * nt / t_co / 1e9, 2),
           "alone_ms": [round(g_alone, 3), round(t_alone, 3)], "co_ms": [round(g_co, 3), round(t_co, 3)],
           # 1.0 = the two ran fully side by side at their alone rates; 0 = serialised
           "overlap": round((g_alone + t_alone - max(g_co, t_co)) / max(min(g_alone, t_alone), 1e-9), 3)}
    print(name, json.dumps(out), flush=True)
    return out


def main():
    res = {"shape": [M, N, K], "triad_floats": NF}
    # calibrate loop counts to ~15 ms alone on the full chip
    full_g, full_t = S(), S()
    timed([(full_g.stream, lambda s: enqueue_gemm(s, 10))])            # warm-up (first launches)
    timed([(full_t.stream, lambda s: enqueue_triad(s, 4))])
    tg = timed([(full_g.stream, lambda s: enqueue_gemm(s, 10))])[0] / 10
    tt = timed([(full_t.stream, lambda s: enqueue_triad(s, 4))])[0] / 4
    ng, nt = max(4, int(15 / tg)), max(2, int(15 / tt))
    res["per_call_ms"] = {"gemm": round(tg, 4), "triad": round(tt, 4)}
    res["loops"] = {"gemm": ng, "triad": nt}
    res["full_share"] = case("full_share", full_g, full_t, ng, nt)
    res["prio_gemm_high"] = case("prio_gemm_high", S(priority=-1), S(), ng, nt)
    res["prio_triad_high"] = case("prio_triad_high", S(), S(priority=-1), ng, nt)
    for gu, tu in (((0, 6), (6, 8)), ((0, 4), (4, 8)), ((0, 3), (3, 8)), ((0, 2), (2, 8))):
        res[f"masked_g{gu}_t{tu}"] = case(f"masked g{gu} t{tu}", S(gu), S(tu), ng, nt, gbudget=(gu[1] - gu[0]) * 32)
    for tu in ((1, 8), (2, 8), (3, 8), (4, 8)):     # only the stream kernel confined; GEMM may use every CU
        res[f"triad_only_masked_t{tu}"] = case(f"triad-only masked t{tu}", S(), S(tu), ng, nt)
    if os.environ.get("PROBE_SHORT"):
        os.makedirs("gpurun_out", exist_ok=True)
        json.dump(res, open("gpurun_out/contention.json", "w"), indent=1)
        return
    # triad launch shape under full sharing
    sweep = {}
    for v, nb in ((6, 0), (3, 256), (3, 512), (3, 1024), (4, 256), (4, 512), (2, 2048)):
        hip.set_triad_variant(v)
        sweep[f"v{v}_b{nb}"] = case(f"triad v{v} b{nb}", full_g, full_t, ng, nt, tblocks=nb)
    hip.set_triad_variant(6)
    res["triad_sweep"] = sweep
    tiles = {}
    for t in (1, 4, 6, 10):
        hip.set_gemm_tile(t)
        tiles[f"tile{t}"] = case(f"gemm tile {t}", full_g, full_t, ng, nt)
    hip.set_gemm_tile(0)
    res["gemm_tiles"] = tiles
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/contention.json", "w"), indent=1)


if __name__ == "__main__":
    main()
