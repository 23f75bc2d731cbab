"""Calibrate rocprofv3's FETCH_SIZE on the GEMMs' load path.

Round 5 turned FETCH_SIZE into HBM read bytes with a x2 factor fitted on the triad's 16-B
non-temporal loads only, and applied it to the GEMMs, whose operands arrive through
global_load_lds.  Here every group has KNOWN compulsory bytes:

  gemm8ph_1tile   M = N = 256, K = 16384, the 8-phase 256x256 kernel: ONE workgroup, so each
                  operand byte is fetched exactly once (A + B = 16 MiB per launch)
  gemm128_1tile   M = N = 128, K = 16384, the 128x128 kernel: one workgroup (8 MiB)
  gemm8ph_bench   2048 x 2048 x 2048 with the bench's 64-CU share tiles (re-fetch across XCDs)
  gemm128_bench   1024 x 1536 x 1536 with share tiles (a mobilenet GEMM)
  triad_nt        64 Mi floats, non-temporal 4x (the bench's variant): 512 MiB read, 256 written
  triad_cached    the same with plain loads / stores

A marker kernel (xcd_probe_kernel) precedes each group; tools/fetch_cal_summary.py splits the
counter CSV at the markers and sets counted bytes against compulsory bytes.
Run: rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -o run -- python3 tools/fetch_cal.py <dir>
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

REPS = 10


def main(out_dir: str) -> None:
    h = _native.hip(required=True)
    torch.cuda.set_device(0)
    mk = torch.zeros(8, dtype=torch.int32, device="cuda")

    def marker() -> None:
        torch.cuda.synchronize()
        h.xcd_probe(mk.data_ptr(), 8, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()

    def operands(M, N, K):
        a = (torch.rand(M, K, device="cuda") - 0.5).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda") - 0.5).to(torch.bfloat16)
        return a, bt, torch.empty(M, N, device="cuda", dtype=torch.bfloat16), torch.zeros(N, device="cuda")

    groups = []
    specs = [("gemm8ph_1tile", 256, 256, 16384, 10, 0), ("gemm128_1tile", 128, 128, 16384, 1, 0),
             ("gemm8ph_bench", 2048, 2048, 2048, 0, 64), ("gemm128_bench", 1024, 1536, 1536, 0, 64)]
    ops = [(name, operands(M, N, K), (M, N, K), tile, budget) for name, M, N, K, tile, budget in specs]
    n = 64 << 20
    x, y, z = (torch.ones(n, device="cuda") for _ in range(3))
    torch.cuda.synchronize()
    for name, (a, bt, c, bias), (M, N, K), tile, budget in ops:
        h.set_gemm_tile(tile)
        t = h.pick_gemm_tile(M, N, budget)
        marker()
        for _ in range(REPS):
            loadgen.gemm(a, bt, out=c, bias=bias, relu=True, cu_budget=budget)
        groups.append({"name": name, "M": M, "N": N, "K": K, "tile": t, "budget": budget,
                       "launches": REPS, "compulsory_read": 2.0 * (M + N) * K * REPS,
                       "compulsory_write": 2.0 * M * N * REPS})
    h.set_gemm_tile(0)
    for name, variant in (("triad_nt", 3), ("triad_cached", 1)):
        h.set_triad_variant(variant)
        marker()
        for _ in range(REPS):
            loadgen.triad(x, y, z, 1.0001)
        groups.append({"name": name, "variant": variant, "launches": REPS,
                       "compulsory_read": 8.0 * n * REPS, "compulsory_write": 4.0 * n * REPS})
    h.set_triad_variant(6)
    marker()
    os.makedirs(out_dir, exist_ok=True)
    json.dump({"groups": groups}, open(os.path.join(out_dir, "groups.json"), "w"), indent=1)
    print("fetch_cal groups:", [g["name"] for g in groups], flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fetch_cal")
