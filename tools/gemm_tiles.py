"""GEMM tile study on the MI355X: every tile variant on every catalog GEMM shape (plus
4096^3 / 8192^3) in isolation, and the aggregate throughput of the catalog mix run as
4 concurrent pods (4 non-blocking streams, like the bench's Burstable pods) per tile
policy.  Interleaved rounds in one process; writes gpurun_out/gemm_tiles.json."""
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

TILES = (1, 2, 3, 4, 5, 6, 7, 8, 9)


def t_ms(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def operands(M, N, K):
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    return a, bt, torch.empty(M, N, device="cuda", dtype=torch.bfloat16), torch.zeros(N, device="cuda")


def main():
    h = _native.hip()
    out = {"isolated": [], "concurrent": []}
    shapes = sorted({(o.M, o.N, o.K) for w in W.CATALOG.values() for o in w.ops if o.kind == "gemm"})
    shapes += [(4096, 4096, 4096), (8192, 8192, 8192)]
    if os.environ.get("GEMM_TILES_CONCURRENT_ONLY"):
        shapes = []
    for (M, N, K) in shapes:
        a, bt, c, bias = operands(M, N, K)
        res = {}
        for rnd in range(2):
            for tile in TILES:
                h.set_gemm_tile(tile)
                tf = 2 * M * N * K / t_ms(lambda: loadgen.gemm(a, bt, out=c, bias=bias, relu=True)) / 1e9
                res[tile] = max(res.get(tile, 0), tf)
        h.set_gemm_tile(0)
        th = t_ms(lambda: torch.relu(torch.addmm(bias.to(torch.bfloat16), a, bt.T)))
        row = {"shape": [M, N, K], "auto": h.pick_gemm_tile(M, N), "torch_tflops": round(2 * M * N * K / th / 1e9, 1),
               "tile_tflops": {str(k): round(v, 1) for k, v in res.items()}}
        out["isolated"].append(row)
        print(row, flush=True)
        del a, bt, c, bias
    # concurrent catalog mix: 4 streams, each a random sequence of catalog GEMMs
    rng = random.Random(0)
    names = [n for n in W.NAMES if any(o.kind == "gemm" for o in W.CATALOG[n].ops)]
    bufs = {}
    for n in names:
        for o in W.CATALOG[n].ops:
            if o.kind == "gemm" and (o.M, o.N, o.K) not in bufs:
                bufs[(o.M, o.N, o.K)] = operands(o.M, o.N, o.K)
    seqs = [[(o.M, o.N, o.K) for n in rng.choices(names, k=24) for o in W.CATALOG[n].ops if o.kind == "gemm"]
            for _ in range(4)]
    streams = [torch.cuda.Stream() for _ in range(4)]
    flops = sum(2 * M * N * K for s in seqs for (M, N, K) in s)

    budget = {"b": 0}

    bias16 = {k: v[3].to(torch.bfloat16) for k, v in bufs.items()}

    def run_mix():
        for st, seq in zip(streams, seqs):
            with torch.cuda.stream(st):
                for (M, N, K) in seq:
                    a, bt, c, bias = bufs[(M, N, K)]
                    if budget["b"] < 0:       # hipBLASLt (torch.addmm) + separate ReLU
                        torch.relu_(torch.addmm(bias16[(M, N, K)], a, bt.T, out=c))
                    else:
                        loadgen.gemm(a, bt, out=c, bias=bias, relu=True, stream=st, cu_budget=budget["b"])
        for st in streams:
            torch.cuda.current_stream().wait_stream(st)
    for rnd in range(3):
        for tile in ("torch", "budget64", "budget64_8ph", 0) + (() if os.environ.get("GEMM_TILES_CONCURRENT_ONLY") else TILES):
            budget["b"] = {"torch": -1, "budget64": 64, "budget64_8ph": 64}.get(tile, 0)
            h.set_gemm_tile(tile if isinstance(tile, int) else 0)
            h.set_gemm_policy(1 if tile == "budget64_8ph" else 0)
            ms = t_ms(run_mix, iters=5, warm=1)
            if rnd:
                out["concurrent"].append({"tile": tile, "round": rnd, "tflops": round(flops / ms / 1e9, 1)})
                print(out["concurrent"][-1], flush=True)
    h.set_gemm_tile(0)
    h.set_gemm_policy(1)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/gemm_tiles.json", "w"), indent=1)


if __name__ == "__main__":
    main()
