"""Kernel microbenchmarks on the MI355X: triad variants x grid sizes, and the MFMA GEMM
on every GEMM shape of the workload catalog vs torch.matmul (hipBLASLt).
Interleaved rounds in one process (guide §5.4 rule 24); writes gpurun_out/kernel_bench.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402


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


def main():
    h = _native.hip()
    out = {"triad": [], "gemm": []}
    for nf in (1024 * 16384, 4096 * 16384):
        x, y, z = (torch.rand(nf, device="cuda") for _ in range(3))
        ref = y + 1.5 * z
        tt = t_ms(lambda: torch.add(y, z, alpha=1.5, out=x))
        out["triad"].append({"n": nf, "variant": "torch", "tbps": 12 * nf / tt / 1e9})
        for rnd in range(2):
            for v in range(6):
                h.set_triad_variant(v)
                for blocks in (1024, 2048, 4096, 8192):
                    ms = t_ms(lambda: loadgen.triad(x, y, z, 1.5, blocks=blocks))
                    if rnd == 1:
                        out["triad"].append({"n": nf, "variant": v, "blocks": blocks, "tbps": 12 * nf / ms / 1e9})
                loadgen.triad(x, y, z, 1.5)
                torch.cuda.synchronize()
                assert torch.allclose(x, ref), v
        h.set_triad_variant(6)
    shapes = sorted({(o.M, o.N, o.K) for w in W.CATALOG.values() for o in w.ops if o.kind == "gemm"})
    for (M, N, K) in shapes:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        bias = torch.zeros(N, device="cuda")
        tiles = {}
        for tile in (1, 2, 3):
            h.set_gemm_tile(tile)
            tiles[tile] = 2 * M * N * K / t_ms(lambda: loadgen.gemm(a, bt, out=c, bias=bias, relu=True)) / 1e9
        h.set_gemm_tile(0)
        ours = t_ms(lambda: loadgen.gemm(a, bt, out=c, bias=bias, relu=True))
        th = t_ms(lambda: torch.relu(torch.addmm(bias.to(torch.bfloat16), a, bt.T)))
        out["gemm"].append({"shape": [M, N, K], "auto_tile": h.pick_gemm_tile(M, N), "ours_us": ours * 1e3,
                            "torch_us": th * 1e3, "ours_tflops": 2 * M * N * K / ours / 1e9,
                            "torch_tflops": 2 * M * N * K / th / 1e9,
                            "tile_tflops": {str(k): round(v, 1) for k, v in tiles.items()}})
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/kernel_bench.json", "w"), indent=1)
    best = {}
    for r in out["triad"]:
        k = r["n"]
        if r["variant"] != "torch" and (k not in best or r["tbps"] > best[k]["tbps"]):
            best[k] = r
    print("best triad", best)
    print("torch triad", [r for r in out["triad"] if r["variant"] == "torch"])
    for g in out["gemm"]:
        print(g)


if __name__ == "__main__":
    main()
