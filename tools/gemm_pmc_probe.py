"""Lone 8192^3 bf16 GEMM: this framework's 8-phase kernel and hipBLASLt (torch.matmul), N
launches each, for a rocprofv3 counter / kernel-trace comparison (tools/gpu_gemm_pmc.sh).

    python tools/gemm_pmc_probe.py [M N K] [iters]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402


def main() -> None:
    M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (8192, 8192, 8192)
    iters = int(sys.argv[4]) if len(sys.argv) >= 5 else 10
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    h = _native.hip(required=True)
    tile = int(os.environ.get("GEMM_TILE", "0"))      # 0: the picker's choice
    picked = h.pick_gemm_tile(M, N, 0)
    h.set_gemm_tile(tile)
    print(f"tile {tile} (picker: {picked}, split-K {h.pick_split_k(M, N, K, 0)})", flush=True)
    for _ in range(3):                      # warm both paths (and the clocks)
        loadgen.gemm(a, bt, out=c)
        torch.matmul(a, bt.t())
    torch.cuda.synchronize()
    for name, fn in (("ours", lambda: loadgen.gemm(a, bt, out=c)), ("hipblaslt", lambda: torch.matmul(a, bt.t()))):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        print(f"{name} {M}x{N}x{K}: {ms:.3f} ms {2.0 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
