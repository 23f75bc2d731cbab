"""A/B of a 0/1 GEMM launch knob of the native module (default set_wide_epilogue; argv[1] names
another, e.g. set_xcd_blocks) on the catalog GEMM shapes: each shape alone (auto tile, whole
chip) and the bench's co-run setting (4 streams, every pod's GEMMs with a 64-CU budget),
interleaved rounds in one process, uniform [-1, 1) operands, bias + ReLU.  Lone big shapes
(4096^3, 8192^3, 8192x8192x2048) are included with argv[2] = "big"."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402


def main():
    h = _native.hip(required=True)
    knob = sys.argv[1] if len(sys.argv) > 1 else "set_wide_epilogue"
    setk = getattr(h, knob)
    shapes = sorted({(o.M, o.N, o.K) for w in W.CATALOG.values() for o in w.ops if o.kind == "gemm"})
    big = [(4096, 4096, 4096), (8192, 8192, 8192), (8192, 8192, 2048)] if "big" in sys.argv[2:] else []
    bufs = {}
    for (M, N, K) in shapes + big:
        bufs[(M, N, K)] = ((torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16),
                           (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16),
                           torch.randn(N, device="cuda"), torch.empty(M, N, device="cuda", dtype=torch.bfloat16))
    streams = [torch.cuda.Stream() for _ in range(4)]

    def lone(shape, reps=20):
        a, bt, b, c = bufs[shape]
        for _ in range(3):
            loadgen.gemm(a, bt, out=c, bias=b, relu=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            loadgen.gemm(a, bt, out=c, bias=b, relu=True)
        e1.record()
        torch.cuda.synchronize()
        M, N, K = shape
        return 2 * M * N * K * reps / (e0.elapsed_time(e1) / 1e3) / 1e12

    def mix(reps=4):
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fl = 0.0
        for r in range(reps):
            for i, shape in enumerate(shapes):
                a, bt, b, c = bufs[shape]
                s = streams[i % 4]
                loadgen.gemm(a, bt, out=c, bias=b, relu=True, stream=s, cu_budget=64)
                fl += 2.0 * shape[0] * shape[1] * shape[2]
        for s in streams:
            torch.cuda.current_stream().wait_stream(s)
        e1.record()
        torch.cuda.synchronize()
        return fl / (e0.elapsed_time(e1) / 1e3) / 1e12

    res = {"lone": {}, "mix": {0: [], 1: []}}
    for rnd in range(3):
        for w in (0, 1):
            setk(w)
            res["mix"][w].append(round(mix(), 1))
            for shape in shapes + big:
                res["lone"].setdefault(str(shape), {0: [], 1: []})[w].append(round(lone(shape), 1))
    setk(1)
    summ = {"mix_tflops": {str(w): sorted(v)[1] for w, v in res["mix"].items()},
            "lone_tflops_median": {k: {str(w): sorted(v)[1] for w, v in d.items()} for k, d in res["lone"].items()}}
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump({"knob": knob, "raw": res, "summary": summ},
              open(f"gpurun_out/{knob.replace('set_', '')}_mix.json", "w"), indent=1)
    print(json.dumps(summ))


if __name__ == "__main__":
    main()
