"""Lone stream-triad HBM rate per kernel variant / cache policy (256 MiB arrays, HIP events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

h = _native.hip(required=True)
n = 64 << 20
x, y, z = (torch.ones(n, device="cuda") for _ in range(3))
for v, aux in ((3, 2), (5, 2), (5, 0), (5, 18), (5, 19), (5, 3), (5, 16)):
    h.set_triad_variant(v)
    h.set_triad_aux(aux)
    for _ in range(3):
        loadgen.triad(x, y, z, 1.0001)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        loadgen.triad(x, y, z, 1.0001)
    e1.record()
    torch.cuda.synchronize()
    print(f"variant {v} aux {aux:2d}: {12.0 * n * 20 / (e0.elapsed_time(e1) / 1e3) / 1e12:.2f} TB/s", flush=True)
h.set_triad_variant(6)
h.set_triad_aux(2)
