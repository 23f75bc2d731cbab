"""bf16 vs fp8 (block-scaled MFMA) GEMM throughput on one MI355X, HIP-event timed.

    python tools/fp8_bench.py [--out gpurun_out/fp8_bench.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/fp8_bench.json")
    a = ap.parse_args()
    rows = []
    for (M, N, K) in [(4096, 4096, 4096), (8192, 8192, 8192), (4096, 2048, 2048), (2048, 4096, 8192)]:
        x = torch.randn(M, K, device="cuda")
        w = torch.randn(N, K, device="cuda")
        xb, wb = x.to(torch.bfloat16), w.to(torch.bfloat16)
        x8, w8 = x.to(loadgen.FP8), w.to(loadgen.FP8)
        ob = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        o8 = torch.empty_like(ob)
        fl = 2.0 * M * N * K
        t_b = timed(lambda: loadgen.gemm(xb, wb, out=ob))
        t_8 = timed(lambda: loadgen.gemm_fp8(x8, w8, out=o8))
        t_t = timed(lambda: torch.matmul(xb, wb.T))
        r = {"M": M, "N": N, "K": K, "bf16_tflops": round(fl / t_b / 1e12, 1),
             "fp8_tflops": round(fl / t_8 / 1e12, 1), "torch_bf16_tflops": round(fl / t_t / 1e12, 1)}
        print(json.dumps(r), flush=True)
        rows.append(r)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
