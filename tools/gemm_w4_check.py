"""Tile 14 (the 4-wave 256 x 256 kernel with AGPR-tied inline-asm MFMAs, 64-deep operand tiles in
a 5-slot LDS ring) on MI355X: numerics
against an fp32 reference, then wall-clock TF/s next to tile 10 (the 8-phase kernel) and
hipBLASLt (torch.matmul) on the lone shapes.

    python tools/gemm_w4_check.py [iters]

Every check runs before any timing; a mismatch exits 1 before the perf loop.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

CHECK = [(256, 256, 128, False, False), (512, 768, 256, True, True), (1024, 2048, 640, False, True),
         (2048, 1024, 1024, True, False), (4096, 4096, 4096, False, False), (512, 768, 256, False, False),
         (2048, 1024, 1024, False, True), (1024, 2048, 640, True, False)]
PERF = [(8192, 8192, 8192), (4096, 4096, 4096), (4096, 8192, 4096), (8192, 8192, 2048)]


def check(h, tile: int) -> bool:
    ok = True
    torch.manual_seed(0)
    for M, N, K, relu, use_bias in CHECK:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        bias = torch.randn(N, device="cuda") if use_bias else None
        ref = a.float() @ bt.float().t()
        if bias is not None:
            ref = ref + bias
        if relu:
            ref = torch.relu(ref)
        h.set_gemm_tile(tile)
        out = loadgen.gemm(a, bt, bias=bias, relu=relu)
        torch.cuda.synchronize()
        err = (out.float() - ref).abs().max().item()
        tol = 0.02 * ref.abs().max().item() + 0.05
        print(f"check tile {tile} {M}x{N}x{K} relu={relu} bias={use_bias}: max err {err:.4f} (tol {tol:.3f})", flush=True)
        ok &= err <= tol
    return ok


def perf(h, iters: int) -> None:
    for M, N, K in PERF:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        arms = {"tile10": 10, "tile14": 14}
        for rnd in range(3):                 # interleaved rounds
            for name, fn in [*((n, t) for n, t in arms.items()), ("hipblaslt", None)]:
                if fn is None:
                    run = lambda: torch.matmul(a, bt.t())  # noqa: E731
                else:
                    h.set_gemm_tile(fn)
                    run = lambda: loadgen.gemm(a, bt, out=c)  # noqa: E731
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / iters
                print(f"round {rnd} {name} {M}x{N}x{K}: {ms:.4f} ms {2.0 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)


def main() -> None:
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    h = _native.hip(required=True)
    try:
        if not all([check(h, t) for t in (14, 15, 16)]):
            print("NUMERICS FAILED", flush=True)
            sys.exit(1)
        perf(h, iters)
    finally:
        h.set_gemm_tile(0)


if __name__ == "__main__":
    main()
