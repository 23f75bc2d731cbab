"""XCD-confinement probe (one MI355X): would a software QPX partition -- each co-running pod's
kernels confined to its own 2 XCDs, so its GEMM operand strips live in 2 L2s instead of 8 --
beat full sharing?

  1. dispatch check: block b runs on XCD b % 8 (xcd_probe_kernel reads HW_REG_XCC_ID; in a
     fresh process -- later launches rotate which XCD takes block 0);
  2. numerics: confined 8-phase GEMM and stream kernel vs the unconfined results (bit-exact);
  3. stream-kernel HBM rate confined to 1 / 2 / 4 / 8 XCDs, and 4 confined streams at once;
  4. the bench's 4-pod pattern: 2 GEMM pods + 2 stream pods on 4 streams, full sharing
     (today's Burstable pods, 64-CU budget) vs each pod confined to its own XCD pair.
Writes gpurun_out/xcd_confine.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

h = _native.hip(required=True)
dev = torch.device("cuda", 0)
PAIRS = [0x03, 0x0C, 0x30, 0xC0]


def timed(jobs):
    """jobs: [(stream, fn)], all started together; returns ms of the slowest."""
    torch.cuda.synchronize()
    start = torch.cuda.Event(enable_timing=True)
    side = torch.cuda.Stream()
    start.record(side)
    ends = []
    for st, fn in jobs:
        st.wait_event(start)
        with torch.cuda.stream(st):
            fn(st)
        e = torch.cuda.Event(enable_timing=True)
        e.record(st)
        ends.append(e)
    torch.cuda.synchronize()
    return [start.elapsed_time(e) for e in ends]


def main():
    out = {}
    # 1. dispatch mapping
    ids = torch.full((8192,), -1, dtype=torch.int32, device=dev)
    h.xcd_probe(ids.data_ptr(), 8192, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ids = ids.cpu()
    ok = bool((ids == torch.arange(8192) % 8).all())
    out["block_on_xcd_b_mod_8"] = ok
    print("block b on XCD b % 8:", ok, ids[:16].tolist(), flush=True)
    if not ok:
        json.dump(out, open("gpurun_out/xcd_confine.json", "w"), indent=1)
        return
    # 2. numerics
    h.set_gemm_tile(10)
    M, N, K = 4096, 2560, 2560
    a = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    bt = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
    bias = torch.randn(N, device=dev)
    ref = loadgen.gemm(a, bt, bias=bias, relu=True)
    n = 4096 * 16384
    x, y, z = (torch.rand(n, device=dev) for _ in range(3))
    tref = torch.empty_like(x)
    loadgen.triad(tref, y, z, 1.0001)              # unconfined kernel (fma rounding, not torch's)
    for m in (0x03, 0x0C, 0x0F, 0x01):
        h.set_xcd_mask(m)
        got = loadgen.gemm(a, bt, bias=bias, relu=True)
        loadgen.triad(x, y, z, 1.0001)
        torch.cuda.synchronize()
        assert torch.equal(got, ref), hex(m)
        assert torch.equal(x, tref), hex(m)
    h.set_xcd_mask(0)
    out["numerics"] = "bit-exact for masks 0x03 0x0C 0x0F 0x01"
    print(out["numerics"], flush=True)
    # 3. stream rate confined
    st = [torch.cuda.Stream() for _ in range(4)]
    rates = {}
    for k, m in ((1, 0x01), (2, 0x03), (4, 0x0F), (8, 0)):
        h.set_xcd_mask(m)
        ms = timed([(st[0], lambda s: [loadgen.triad(x, y, z, 1.0001, stream=s) for _ in range(10)])])[0]
        rates[k] = round(12.0 * n * 10 / ms / 1e9, 2)
    h.set_xcd_mask(0)
    out["triad_tbps_on_k_xcds"] = rates
    print("triad TB/s on k XCDs", rates, flush=True)
    xs = [tuple(torch.rand(n // 4, device=dev) for _ in range(3)) for _ in range(4)]

    def tri_pod(i, mask):
        def fn(s):
            h.set_xcd_mask(mask)
            for _ in range(10):
                loadgen.triad(*xs[i], 1.0001, stream=s)
        return fn
    ms = max(timed([(st[i], tri_pod(i, PAIRS[i])) for i in range(4)]))
    h.set_xcd_mask(0)
    full = max(timed([(st[i], tri_pod(i, 0)) for i in range(4)]))
    out["four_streams_tbps"] = {"confined_pairs": round(12.0 * n * 10 / ms / 1e9, 2),
                                "full_share": round(12.0 * n * 10 / full / 1e9, 2)}
    print("4 concurrent streams", out["four_streams_tbps"], flush=True)
    # 4. 2 GEMM pods + 2 stream pods
    ga = [((torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16),
           ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16),
           torch.empty(M, N, device=dev, dtype=torch.bfloat16)) for _ in range(2)]

    def gemm_pod(i, mask, reps):
        def fn(s):
            h.set_xcd_mask(mask)
            for _ in range(reps):
                loadgen.gemm(ga[i][0], ga[i][1], out=ga[i][2], bias=bias, relu=True, stream=s,
                             cu_budget=0 if mask else 64)
        return fn

    def stream_pod(i, mask, reps):
        def fn(s):
            h.set_xcd_mask(mask)
            for _ in range(reps):
                loadgen.triad(*xs[i], 1.0001, stream=s)
        return fn
    res = {}
    for rnd in range(3):
        for name, masks in (("full_share", (0, 0, 0, 0)), ("confined_pairs", PAIRS)):
            t = timed([(st[0], gemm_pod(0, masks[0], 40)), (st[1], gemm_pod(1, masks[1], 40)),
                       (st[2], stream_pod(2, masks[2], 12)), (st[3], stream_pod(3, masks[3], 12))])
            res.setdefault(name, []).append([round(v, 3) for v in t])
            h.set_xcd_mask(0)
    out["two_gemm_two_stream_pods_ms"] = res
    out["summary"] = {k: min(max(r) for r in v) for k, v in res.items()}
    print("2 GEMM + 2 stream pods, per-pod ms", json.dumps(res), flush=True)
    print("slowest pod, best of 3:", out["summary"], flush=True)
    h.set_gemm_tile(0)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/xcd_confine.json", "w"), indent=1)


if __name__ == "__main__":
    main()
