"""Benchmark entry point (driver contract): `python bench.py --gpus N --steps K --warmup W`.

Runs the pod-arrival scheduling benchmark (k8s_gpu_scheduler_amd.parallel.podbench): one
process per GPU (torchrun sets RANK/LOCAL_RANK/WORLD_SIZE), rank 0 hosts the control
plane (apiserver + scheduler + GPU plugin), every rank executes its GPU's pods on
CU-masked streams with the native MFMA/HBM kernels, placements and telemetry move over
RCCL.  Prints ONE JSON line on rank 0 (metric/config from BASELINE.json).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from k8s_gpu_scheduler_amd.parallel.podbench import main  # noqa: E402

if __name__ == "__main__":
    main()
