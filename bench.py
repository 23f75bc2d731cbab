"""Benchmark entry point (driver contract): `python bench.py --gpus N --steps K --warmup W`.

Runs the pod-arrival scheduling benchmark (k8s_gpu_scheduler_amd.parallel.podbench): one
process per GPU (torchrun sets RANK/LOCAL_RANK/WORLD_SIZE), rank 0 hosts the control
plane (apiserver + scheduler + GPU plugin), every rank executes its GPU's pods on
CU-masked streams with the native MFMA/HBM kernels, placements and telemetry move over
RCCL.  Prints ONE JSON line on rank 0 (metric/config from BASELINE.json).
"""
import os
import sys

# HIP hardware queues per process (HIP's default, and the GPU box's environment, is 4): the 4
# pod streams, the control stream, the null stream and RCCL's streams each need a queue of
# their own -- pod streams that share a queue run back to back instead of side by side
# (interleaved A/B on MI355X: 4 -> 8 queues = +2.9 % pods/s, profiles/archive/r02_hwq_ab.txt; pod
# start/end events: tools/concurrency_probe.py), and an RCCL stream sharing a pod's queue
# would hold the per-epoch placement broadcast behind that pod's queued kernels.  HIP creates
# a queue per stream only up to this limit, so headroom costs nothing while the process has
# fewer streams.  Raised (never lowered) before HIP initialises; GPUSCHED_HW_QUEUES overrides.
_q = int(os.environ.get("GPUSCHED_HW_QUEUES", "16"))
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < _q <= 32:
    os.environ["GPU_MAX_HW_QUEUES"] = str(_q)

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from k8s_gpu_scheduler_amd.parallel.podbench import main  # noqa: E402

if __name__ == "__main__":
    main()
