"""Co-run launch-policy study: epochs of 4 co-running pods (random catalog workloads,
2 CU units each, Burstable) through the real DeviceExecutor, per policy
(GEMM tile by pod share vs whole chip; stream-kernel grid size).  Interleaved rounds in
one process; writes gpurun_out/pod_mix.json."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.models import workloads as W  # noqa: E402
from k8s_gpu_scheduler_amd.parallel.executor import DeviceExecutor, PodRun  # noqa: E402

POLICIES = [(False, 0), (True, 0), (True, 4096), (True, 2048), (True, 1024), (True, 512), (False, 1024)]


def main():
    ex = DeviceExecutor(0)
    rng = random.Random(1)
    weights = [1.0 / (1 + (i % 6)) for i in range(len(W.NAMES))]
    epochs = [[PodRun(4 * e + i, rng.choices(W.NAMES, weights)[0], 2 * i, 2, 20, masked=False) for i in range(4)]
              for e in range(12)]
    ex.warm([PodRun(0, wl, u, 2, 1, masked=False) for wl in W.NAMES for u in (0, 2, 4, 6)])
    res = {}
    for rnd in range(3):
        for pol in POLICIES:
            ex.gemm_share, ex.triad_blocks = pol
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for ep in epochs:
                ex.launch_epoch(ep)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / len(epochs) * 1e3
            if rnd:
                res.setdefault(str(pol), []).append(round(ms, 3))
        print(rnd, {k: v[-1] for k, v in res.items()} if rnd else "warm", flush=True)
    out = {k: {"ms_per_epoch": v, "best": min(v)} for k, v in res.items()}
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/pod_mix.json", "w"), indent=1)
    for k, v in sorted(out.items(), key=lambda kv: kv[1]["best"]):
        print(k, v)
    ex.close()


if __name__ == "__main__":
    main()
