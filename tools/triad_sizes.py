"""Lone stream-triad bandwidth per working-set size for the non-temporal (3) and write-through
(8) store variants: the bench's triads stream 3 x 64 / 128 / 256 MiB (batch 1024 / 2048 / 4096),
the smaller ones within reach of the 256 MiB Infinity Cache across a pod's 20 iterations."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402


def main() -> None:
    h = _native.hip(required=True)
    res = []
    for n in (16 << 20, 32 << 20, 64 << 20):
        x, y, z = (torch.ones(n, device="cuda") for _ in range(3))
        for rnd in range(2):
            for v in (3, 8):
                h.set_triad_variant(v)
                for _ in range(3):
                    loadgen.triad(x, y, z, 1.0001)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    loadgen.triad(x, y, z, 1.0001)
                e1.record()
                torch.cuda.synchronize()
                r = {"mib_per_array": n * 4 >> 20, "variant": v,
                     "tbps": round(12.0 * n * 20 / (e0.elapsed_time(e1) / 1e3) / 1e12, 3)}
                if rnd:
                    res.append(r)
                    print(json.dumps(r), flush=True)
        del x, y, z
    h.set_triad_variant(6)
    json.dump(res, open("gpurun_out/triad_sizes.json", "w"), indent=1)


if __name__ == "__main__":
    main()
