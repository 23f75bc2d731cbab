"""Control-plane throughput at N GPUs (CPU only): ms to schedule one epoch of N x 4 pods."""
import sys
import time

sys.path.insert(0, ".")
from k8s_gpu_scheduler_amd.parallel.podbench import ControlPlane  # noqa: E402

for n in (1, 2, 4, 8):
    cp = ControlPlane(n, 4, 20, 0)
    for _ in range(10):
        cp.finish_live()
        cp.schedule_epoch()
    t = time.perf_counter()
    for _ in range(100):
        cp.finish_live()
        cp.schedule_epoch()
    dt = (time.perf_counter() - t) / 100
    print(f"gpus={n} pods/epoch={4 * n} ms/epoch={dt * 1e3:.2f} ms/pod={dt * 1e3 / (4 * n):.3f}", flush=True)
