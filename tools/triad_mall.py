"""Infinity-Cache-aware streaming: a pod re-streams the same triad arrays every query batch.
Time 20 sweeps of two triads (a mobilenet-1024-like pod: 2 x 16.7M floats, 402 MB working set)
with a cached prefix of P bytes per triad (rest non-temporal), alone and as 4 concurrent pods
on 4 streams (1.6 GB total), for several prefix budgets.  Writes gpurun_out/triad_mall.json."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import torch  # noqa: E402

from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

NF = int(os.environ.get("TRIAD_MALL_FLOATS", str(1024 * 16384)))
SWEEPS = 20


def pod_bufs():
    return [tuple(torch.ones(NF, device="cuda") for _ in range(3)) for _ in range(2)]


def run(pods, streams, cached_floats):
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for st in streams:
        st.wait_event(e0)
    for _ in range(SWEEPS):
        for bufs, st in zip(pods, streams):
            for x, y, z in bufs:
                loadgen.triad(x, y, z, 1.0001, stream=st, cached_floats=cached_floats)
    for st in streams:
        e = torch.cuda.Event()
        e.record(st)
        torch.cuda.current_stream().wait_event(e)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    gb = 12.0 * NF * 2 * SWEEPS * len(pods) / 1e9
    return ms, gb / ms


def main():
    out = {"floats_per_triad": NF, "sweeps": SWEEPS, "alone": {}, "four_pods": {}}
    pods = [pod_bufs() for _ in range(4)]
    streams = [torch.cuda.Stream() for _ in range(4)]
    mb = [0, 16, 32, 48, 64, 96, 128]
    for rnd in range(3):
        for p in mb:
            cf = min(NF, int(p * 2**20 / 12) // 4 * 4)          # P MiB of the 3 arrays per triad
            ms, tbps = run(pods[:1], streams[:1], cf)
            out["alone"].setdefault(str(p), []).append(round(tbps, 3))
            cf4 = min(NF, int(p / 4 * 2**20 / 12) // 4 * 4)    # the same MALL budget split over 4 pods
            ms4, tbps4 = run(pods, streams, cf4)
            out["four_pods"].setdefault(str(p), []).append(round(tbps4, 3))
        print(rnd, {k: v[-1] for k, v in out["alone"].items()}, {k: v[-1] for k, v in out["four_pods"].items()},
              flush=True)
    out["note"] = ("effective TB/s = (every byte the triads read + write) / time; alone: one pod's two "
                   "triads with P MiB cached per triad; four_pods: 4 pods on 4 streams with P/4 MiB cached "
                   "per triad each (P = the whole budget per triad index)")
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(out, open("gpurun_out/triad_mall.json", "w"), indent=1)


if __name__ == "__main__":
    main()
