"""Lone large GEMMs: the 8-phase 256x256 kernel under each XCD tile-order setting (XCD-block
order with 2 / 4 / 8 / 16 tile rows per group, and the plain GROUP_M order -- the lone-GEMM
default since round 4, set_lone_plain_order) against hipBLASLt
(torch), interleaved rounds in one process on uniform [-1, 1) operands.
Writes gpurun_out/gemm_xcd_sweep.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 8192, 2048), (4096, 8192, 4096), (2048, 4096, 8192)]
ARMS = os.environ.get("XCD_SWEEP_ARMS", "torch,g2,g4,g8,g16,plain").split(",")
ROUNDS = int(os.environ.get("XCD_SWEEP_ROUNDS", "3"))


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
        ref = (a.float() @ bt.float().T)
        res = {x: [] for x in ARMS}
        for _ in range(ROUNDS):
            for arm in ARMS:
                if arm == "torch":
                    fn = lambda: torch.matmul(a, bt.T, out=c)  # noqa: E731
                else:
                    h.set_gemm_tile(10)
                    h.set_lone_plain_order(1 if arm == "plain" else 0)
                    if arm != "plain":
                        h.set_xcd_blocks(1)
                        h.set_xcd_group(int(arm[1:]))
                    fn = lambda: loadgen.gemm(a, bt, out=c)  # noqa: E731
                res[arm].append(round(2 * M * N * K / t_ms(fn) / 1e9, 1))
                if arm != "torch":
                    err = (c.float() - ref).abs().max().item()
                    assert err < 0.05 * ref.abs().max().item() + 0.5, (arm, err)
        h.set_gemm_tile(0)
        h.set_xcd_blocks(1)
        h.set_xcd_group(4)
        h.set_lone_plain_order(1)
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        row = {"shape": [M, N, K], "median_tflops": med,
               "vs_hipblaslt": {k: round(v / med["torch"], 3) for k, v in med.items() if k != "torch"}}
        out.append(row)
        print(json.dumps(row), flush=True)
        del a, bt, c, ref
    os.makedirs("gpurun_out", exist_ok=True)
    with open(os.environ.get("XCD_SWEEP_OUT", "gpurun_out/gemm_xcd_sweep.json"), "w") as f:
        json.dump({"rounds": ROUNDS, "note": "uniform [-1,1) bf16, bf16 out, no bias/act; median TF/s of interleaved rounds x 20 "
                           "iters; g<k> = XCD-block order with k tile rows per group (default 4), plain = GROUP_M "
                           "order", "results": out}, f, indent=1)


if __name__ == "__main__":
    main()
