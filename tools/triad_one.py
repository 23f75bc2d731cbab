"""One stream-triad configuration, for PMC passes: python triad_one.py <n_floats> <variant> <reps>."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from k8s_gpu_scheduler_amd import _native  # noqa: E402
from k8s_gpu_scheduler_amd.ops import loadgen  # noqa: E402

n, variant, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
_native.hip(required=True).set_triad_variant(variant)
x, y, z = (torch.ones(n, device="cuda") for _ in range(3))
for _ in range(reps):
    loadgen.triad(x, y, z, 1.0001)
torch.cuda.synchronize()
start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
start.record()
for _ in range(reps):
    loadgen.triad(x, y, z, 1.0001)
end.record()
torch.cuda.synchronize()
ms = start.elapsed_time(end) / reps
print(f"triad n={n} variant={variant}: {ms * 1e3:.1f} us, {12 * n / ms / 1e9:.2f} TB/s")
