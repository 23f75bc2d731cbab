"""GPU diagnostics for the native layer (run on the MI355X box via gpurun).

Measures what the scheduler's design relies on:
  1. device query (CUs, arch, HBM)
  2. logical-CU -> XCD mapping under CU masks (probe kernel reads HW_REG_XCC_ID)
  3. MFMA GEMM correctness vs a torch fp32 reference, and TFLOP/s vs torch.matmul
  4. HBM triad bandwidth
  5. fractional sharing: 4 pods on 4 XCD-pair-masked streams vs the same work serially
Writes gpurun_out/diag.json.
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import cumask, loadgen  # noqa: E402
from k8s_gpu_scheduler_amd.plugins.gpu.devices import cu_slice_mask  # noqa: E402


def timed(fn, iters=10, warmup=3, stream=None):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters / 1e3


def main() -> None:
    out = {}
    h = _native.hip()
    out["devices"] = h.query_all()
    print("devices", out["devices"][0], flush=True)
    # 2. XCD map
    out["probe_unmasked"] = cumask.probe_xcd_map(None, 4096)
    out["probe_bits_0_31"] = cumask.probe_xcd_map([0xFFFFFFFF] + [0] * 7, 2048)
    out["probe_bits_0_7"] = cumask.probe_xcd_map([0xFF] + [0] * 7, 2048)
    out["probe_slot_masks"] = cumask.verify_unit_masks(2)
    print("probe", json.dumps(out["probe_slot_masks"])[:800], flush=True)
    # 3. GEMM correctness + speed
    torch.manual_seed(0)
    corr = []
    for (M, N, K) in [(128, 128, 64), (256, 384, 192), (1024, 512, 2048), (2048, 2048, 1024)]:
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        bt = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        c = loadgen.gemm(a, bt, bias=bias, relu=True)
        ref = torch.relu(a.float() @ bt.float().T + bias)
        err = (c.float() - ref).abs().max().item()
        rel = err / ref.abs().max().item()
        corr.append({"shape": [M, N, K], "max_abs_err": err, "rel": rel})
    out["gemm_correctness"] = corr
    print("corr", corr, flush=True)
    perf = []
    for n in (2048, 4096, 8192):
        a = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
        bt = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
        c = torch.empty(n, n, device="cuda", dtype=torch.bfloat16)
        t = timed(lambda: loadgen.gemm(a, bt, out=c), iters=20)
        tt = timed(lambda: torch.matmul(a, bt.T), iters=20)
        perf.append({"n": n, "ours_tflops": 2 * n ** 3 / t / 1e12, "torch_tflops": 2 * n ** 3 / tt / 1e12})
    out["gemm_perf"] = perf
    print("perf", perf, flush=True)
    # 4. triad
    nf = 256 * 1024 * 1024
    x, y, z = (torch.ones(nf, device="cuda") for _ in range(3))
    t = timed(lambda: loadgen.triad(x, y, z, 2.0), iters=10)
    out["triad_tbps"] = 3 * nf * 4 / t / 1e12
    t = timed(lambda: torch.add(y, z, alpha=2.0, out=x), iters=10)
    out["torch_add_tbps"] = 3 * nf * 4 / t / 1e12
    print("triad", out["triad_tbps"], out["torch_add_tbps"], flush=True)
    # 5. masked concurrency
    n = 4096
    a = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
    bt = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
    cs = [torch.empty(n, n, device="cuda", dtype=torch.bfloat16) for _ in range(4)]
    streams = [cumask.MaskedStream(cu_slice_mask(2 * i, 2)) for i in range(4)]
    reps = 10

    def serial():
        for i in range(4):
            for _ in range(reps):
                loadgen.gemm(a, bt, out=cs[i])

    def concurrent():
        ev = torch.cuda.Event()
        ev.record()
        for i, ms in enumerate(streams):
            ms.stream.wait_event(ev)
            for _ in range(reps):
                loadgen.gemm(a, bt, out=cs[i], stream=ms.stream)
        for ms in streams:
            e = torch.cuda.Event()
            e.record(ms.stream)
            torch.cuda.current_stream().wait_event(e)

    def one_quarter():
        for _ in range(reps):
            loadgen.gemm(a, bt, out=cs[0], stream=streams[0].stream)
        e = torch.cuda.Event()
        e.record(streams[0].stream)
        torch.cuda.current_stream().wait_event(e)

    ts = timed(serial, iters=3, warmup=1)
    tc = timed(concurrent, iters=3, warmup=1)
    tq = timed(one_quarter, iters=3, warmup=1)
    fl = 4 * reps * 2 * n ** 3
    out["masked"] = {"serial_full_tflops": fl / ts / 1e12, "concurrent_4x_quarter_tflops": fl / tc / 1e12,
                     "single_quarter_tflops": fl / 4 / tq / 1e12}
    print("masked", out["masked"], flush=True)
    for s in streams:
        s.close()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/diag.json", "w") as f:
        json.dump(out, f, indent=1, default=str)
    print("DIAG OK")


if __name__ == "__main__":
    main()
