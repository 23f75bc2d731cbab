"""Large lone GEMMs (a whole-GPU pod): the default picker (arm 0: 8-phase 256x256, or split-K
when its tiles leave CUs idle), the 256x256 8-phase kernel (tile 9/10) against the
256x256 2-stage (4), the 128x128 (1) and hipBLASLt (torch), interleaved rounds in one
process on uniform [-1, 1) operands.  Writes gpurun_out/gemm_big.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 8192, 2048), (4096, 8192, 4096), (2048, 4096, 8192)]
ARMS = ["torch"] + [int(x) for x in os.environ.get("GEMM_BIG_ARMS", "0,1,10").split(",")]


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
    h = _native.hip(required=True)
    out = []
    for (M, N, K) in SHAPES:
        a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        res = {str(x): [] for x in ARMS}
        for _ in range(3):
            for arm in ARMS:
                if arm == "torch":
                    fn = lambda: torch.matmul(a, bt.T, out=c)  # noqa: E731
                else:
                    h.set_gemm_tile(arm)
                    fn = lambda: loadgen.gemm(a, bt, out=c)  # noqa: E731
                res[str(arm)].append(round(2 * M * N * K / t_ms(fn) / 1e9, 1))
        h.set_gemm_tile(0)
        row = {"shape": [M, N, K], "tflops": {k: {"best": max(v), "median": sorted(v)[1]} for k, v in res.items()}}
        out.append(row)
        print(json.dumps(row), flush=True)
        del a, bt, c
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/gemm_big.json", "w") as f:
        json.dump({"note": "uniform [-1,1) bf16 operands, bf16 out, no bias/act; TF/s best and median of 3 "
                           "interleaved rounds x 20 iters", "results": out}, f, indent=1)


if __name__ == "__main__":
    main()
