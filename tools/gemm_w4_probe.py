"""Where the 4-wave kernel's time goes (timing only): tile 14 with its steady loop's LDS-DMA
dropped (probe 1), its fragment reads dropped (2) or both (3), next to the full kernel, tile 10
and hipBLASLt, interleaved rounds.
Probes 1-3 compute garbage by design.  W4_ARMS=name,name,... selects arms.

    python tools/gemm_w4_probe.py [M N K] [iters]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402


def main() -> None:
    M, N, K = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (8192, 8192, 8192)
    iters = int(sys.argv[4]) if len(sys.argv) >= 5 else 30
    h = _native.hip(required=True)
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    arms = [("tile10", 10, 0), ("tile14", 14, 0), ("w4_no_glds", 14, 1), ("w4_no_reads", 14, 2),
            ("w4_mfma_only", 14, 3), ("hipblaslt", None, 0)]
    if os.environ.get("W4_ARMS"):
        keep = set(os.environ["W4_ARMS"].split(","))
        arms = [a for a in arms if a[0] in keep]
    try:
        for rnd in range(3):
            for name, tile, probe in arms:
                if tile is None:
                    run = lambda: torch.matmul(a, bt.t())  # noqa: E731
                else:
                    h.set_gemm_tile(tile)
                    h.set_w4_probe(probe)
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
    finally:
        h.set_w4_probe(0)
        h.set_gemm_tile(0)


if __name__ == "__main__":
    main()
