"""Small co-run GEMMs on MI355X: the catalog GEMM shapes that a quarter-GPU pod (64-CU budget)
runs on the 128x128 tile family, per tile variant, in the three settings a pod meets:

  one   -- one pod alone on its 64-CU CU-mask slice (a Guaranteed pod next to idle CUs)
  four  -- four pods, each on its own 64-CU slice, all running the shape (a full chip of
           Guaranteed pods: every CU busy, the L2 / MALL shared)
  burst -- four unmasked streams (Burstable pods, the bench's QoS) running the shape

TF/s per setting and the MFMA utilisation it implies against the dense bf16 peak of the CUs the
setting owns (2.5 PF x 64/256 per pod).  Interleaved rounds in one process; writes
gpurun_out/small_gemm_study.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402
from k8s_gpu_scheduler_amd.ops.cumask import MaskedStream  # noqa: E402
from k8s_gpu_scheduler_amd.plugins.gpu.devices import cu_slice_mask  # noqa: E402

PEAK_TF = 2500.0
TILES = [int(t) for t in os.environ.get("SMALL_GEMM_TILES", "1,13,10").split(",")]
REPS = 8


def main() -> None:
    h = _native.hip(required=True)
    shapes = sorted({(o.M, o.N, o.K) for w in W.CATALOG.values() for o in w.ops
                     if o.kind == "gemm" and h.pick_gemm_tile(o.M, o.N, 64) == 1})
    masked = [MaskedStream(cu_slice_mask(2 * i, 2), 0) for i in range(4)]
    plain = [torch.cuda.Stream() for _ in range(4)]
    ops = {}
    for (M, N, K) in shapes:
        ops[(M, N, K)] = [((torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16),
                           ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16),
                           torch.empty(M, N, device="cuda", dtype=torch.bfloat16),
                           torch.zeros(N, device="cuda")) for _ in range(4)]

    def run(shape, streams):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        ev0.record()
        for st in streams:
            st.wait_event(ev0)
        for i, st in enumerate(streams):
            a, bt, c, b = ops[shape][i]
            for _ in range(REPS):
                loadgen.gemm(a, bt, out=c, bias=b, relu=True, stream=st, cu_budget=64)
        for st in streams:
            ev = torch.cuda.Event()
            ev.record(st)
            torch.cuda.current_stream().wait_event(ev)
        ev1.record()
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1)

    res = {}
    for rnd in range(3):
        for shape in shapes:
            M, N, K = shape
            fl = 2.0 * M * N * K * REPS
            for t in TILES:
                h.set_gemm_tile(t)
                try:
                    for name, sts in (("one", [masked[0].stream]), ("four", [m.stream for m in masked]),
                                      ("burst", plain)):
                        ms = run(shape, sts)
                        if rnd == 0:
                            continue
                        tf = fl * len(sts) / (ms / 1e3) / 1e12
                        k = f"{M}x{N}x{K}"
                        cur = res.setdefault(k, {}).setdefault(str(t), {})
                        cur[name] = max(cur.get(name, 0.0), round(tf, 1))
                finally:
                    h.set_gemm_tile(0)
        if rnd:
            print("round", rnd, json.dumps(res), flush=True)
    summary = {}
    for k, per in res.items():
        summary[k] = {t: dict(v, one_mfma_pct=round(100 * v["one"] / (PEAK_TF / 4), 1),
                              four_mfma_pct=round(100 * v["four"] / PEAK_TF, 1)) for t, v in per.items()}
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump({"tiles": TILES, "reps": REPS, "results": summary}, open("gpurun_out/small_gemm_study.json", "w"),
              indent=1)
    for k, per in summary.items():
        print(k, per)
    for m in masked:
        m.close()


if __name__ == "__main__":
    main()
