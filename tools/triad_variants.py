"""Lone HBM bandwidth of each stream-triad variant (native set_triad_variant) on a 768 MB
triad, and the same next to a co-running 8-phase 256x256 GEMM stream (the bench's dominant
GEMM family): TB/s of the triad and TF/s of the GEMM side by side.  Prints JSON lines."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402


def main() -> None:
    h = _native.hip(required=True)
    n = 64 << 20
    x, y, z = (torch.ones(n, device="cuda") for _ in range(3))
    a = (torch.rand(4096, 2048, device="cuda") - 0.5).to(torch.bfloat16)
    bt = (torch.rand(2048, 2048, device="cuda") - 0.5).to(torch.bfloat16)
    c = torch.empty(4096, 2048, device="cuda", dtype=torch.bfloat16)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    res = {}
    for rnd in range(3):
        for v in tuple(int(x) for x in os.environ.get("TRIAD_VARIANTS", "3,5,7").split(",")):
            h.set_triad_variant(v)
            for co in (False, True):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s1)
                for _ in range(10):
                    loadgen.triad(x, y, z, 1.0001, stream=s1)
                e1.record(s1)
                if co:
                    g0.record(s2)
                    for _ in range(40):
                        loadgen.gemm(a, bt, out=c, relu=True, stream=s2, cu_budget=64)
                    g1.record(s2)
                torch.cuda.synchronize()
                tms = e0.elapsed_time(e1)
                r = {"variant": v, "corun": co, "triad_tbps": round(12.0 * n * 10 / (tms / 1e3) / 1e12, 3)}
                if co:
                    gms = g0.elapsed_time(g1)
                    r["gemm_tfs"] = round(2.0 * 4096 * 2048 * 2048 * 40 / (gms / 1e3) / 1e12, 1)
                    r["wall_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
                if rnd:
                    res.setdefault(f"{v}_{int(co)}", []).append(r)
                    print(json.dumps(r), flush=True)
    h.set_triad_variant(6)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/triad_variants.json", "w"), indent=1)


if __name__ == "__main__":
    main()
