"""Phase-split co-run study: do co-running pods overlap HBM streaming with MFMA work better
when each roofline class gets its own CU units?

profiles/r01_overlap_study.json showed the bench's pod mix barely overlaps the two
classes when every pod's kernels share all 256 CUs (full 8.10 ms = GEMM-only 2.86 + triad-only
5.74 - 0.50 per epoch).  Here the executor's `phase_split = k` sends every pod's stream
triads to a stream masked to CU units [0, k) and its GEMMs to one masked to [k, 8) (a unit =
4 CUs on each of the 8 XCDs).  Measured, interleaved per round:
  * triad bandwidth and GEMM rate alone on k units (the per-class scaling curves),
  * the full pod mix at phase_split = 0 (today) and k = 2..6.
Writes gpurun_out/phase_split.json."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402
from k8s_gpu_scheduler_amd.ops.cumask import MaskedStream  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402


def timed(fn, reps=1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


def main():
    out = {"note": __doc__.split("\n")[0]}
    ks = [int(x) for x in os.environ.get("SPLIT_KS", "2,3,4,5,6").split(",")]
    # ---- per-class scaling on k units ------------------------------------------------
    n = 4096 * 16384                       # the largest catalog triad (256 MiB per array)
    x, y, z = (torch.ones(n, device="cuda") for _ in range(3))
    a = torch.randn(4096, 2048, device="cuda").to(torch.bfloat16)
    bt = torch.randn(2048, 2048, device="cuda").to(torch.bfloat16)
    c = torch.empty(4096, 2048, device="cuda", dtype=torch.bfloat16)
    curve = {}
    for k in ([] if os.environ.get("SKIP_CURVE") else range(1, 9)):
        ms = MaskedStream.for_units(0, k)
        tri = timed(lambda: [loadgen.triad(x, y, z, 1.0001, stream=ms.stream) for _ in range(10)]) / 10
        gem = timed(lambda: [loadgen.gemm(a, bt, out=c, relu=True, stream=ms.stream, cu_budget=32 * k)
                             for _ in range(20)]) / 20
        curve[k] = {"triad_tbps": round(12.0 * n / tri / 1e9, 3),
                    "gemm_tflops": round(2.0 * 4096 * 2048 * 2048 / gem / 1e9, 1)}
        ms.close()
        print("units", k, curve[k], flush=True)
    out["per_units"] = curve
    del x, y, z
    # ---- bench pod mix ---------------------------------------------------------------
    ex = DeviceExecutor(0)
    rng = random.Random(1)
    weights = [1.0 / (1 + (i % 6)) for i in range(len(W.NAMES))]
    epochs = [[PodRun(4 * e + i, rng.choices(W.NAMES, weights)[0], 2 * i, 2, 20, masked=False) for i in range(4)]
              for e in range(12)]
    ex.warm([PodRun(0, wl, u, 2, 1, masked=False) for wl in W.NAMES for u in (0, 2, 4, 6)])

    modes = [("base", 0, False, True)] + [(f"op{k}", k, False, True) for k in ks] + \
        [(f"pod{k}", k, True, True) for k in ks] + [("op_nomask", 4, False, False)] + \
        [(f"pod{k}s", k, True, True) for k in ks]
    only = os.environ.get("MODES")
    if only:            # one process per mode: idle extra queues slow every stream
        modes = [m for m in modes if m[0] in only.split(",")]

    def run(mode):
        name, k, by_pod, masks = mode
        ex.phase_split, ex.split_by_pod, ex.split_masks = k, by_pod, masks
        ex.split_shared = name.endswith("s")
        eps = [[PodRun(r.pod_id, r.workload, r.first_unit, r.n_units, r.iters, masked=False) for r in ep]
               for ep in epochs]
        return timed(lambda: [ex.launch_epoch(ep) for ep in eps]) / len(eps)

    if os.environ.get("SKIP_CURVE"):
        out.pop("per_units", None)
    for m in modes:                         # create the split streams outside the timing
        run(m)
    res = {}
    for rnd in range(4):
        for m in modes:
            ms = run(m)
            if rnd:
                res.setdefault(m[0], []).append(round(ms, 3))
        print(rnd, {k: v[-1] for k, v in res.items()}, flush=True)
    out["ms_per_epoch"] = {str(k): {"runs": v, "best": min(v), "median": sorted(v)[len(v) // 2]}
                           for k, v in res.items()}
    ex.phase_split, ex.split_by_pod, ex.split_masks = 0, False, True
    ex.close()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open(f"gpurun_out/phase_split{'_' + only if only else ''}.json", "w"), indent=1)
    print(json.dumps(out["ms_per_epoch"]))


if __name__ == "__main__":
    main()
